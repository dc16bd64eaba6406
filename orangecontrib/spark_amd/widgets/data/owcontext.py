"""Context widget: create the shared Session (reference: widgets/data/spark_context.py:13-78).

``spark.executor.instances`` defaults to ``auto`` = every visible MI355X (the reference's
default cluster is 8 executors, spark_context.py:41); the info line lists the executor
devices, and an executor loss (the pool respawns and rebuilds handles from lineage) is
reported as a warning on this widget."""
from collections import OrderedDict

from orange3_spark_amd.conf import DEFAULTS, SessionConf

from ...utils.gui_param import GuiParam
from ..base import SharedSession
from ..compat import Setting, Widget


class OWSessionContext(SharedSession, Widget):
    priority = 0
    name = "Context"
    description = "Create the shared MI355X session (replaces the Spark/Hive contexts)"
    icon = "../icons/context.svg"
    inputs, outputs = [], []
    saved_gui_params = Setting(OrderedDict())

    def __init__(self, **kw):
        super().__init__(**kw)
        # the reference's order (spark_context.py:31-32,49-58): defaults, then every key the
        # configuration already holds (O3S_CONF_* environment keys), then saved values
        self.conf = SessionConf()
        params = OrderedDict(DEFAULTS)
        for k, v in self.conf.getAll():
            params[k] = v
        if params.get("o3s.session.warmup") == DEFAULTS["o3s.session.warmup"]:
            # the canvas's session is created ahead of its first fit (this widget's action
            # runs on a worker thread): warm every estimator family then (runtime/warmup.py)
            params["o3s.session.warmup"] = "all"
        for k, v in self.saved_gui_params.items():
            params[k] = v
        self.gui_parameters = OrderedDict((k, GuiParam(label=k, default_value=str(v))) for k, v in params.items())

    def set_param(self, key, value):
        if key not in self.gui_parameters:
            self.gui_parameters[key] = GuiParam(label=key, default_value=str(value))
        else:
            self.gui_parameters[key].set_value(value)
        return self

    def create_context(self):
        from orange3_spark_amd import Session
        if self.session is not None:
            self.session.stop()
        conf = SessionConf(loadDefaults=False)
        for key, p in self.gui_parameters.items():
            conf.set(key, p.get_value())
            self.saved_gui_params[key] = p.get_value()
        self.session = Session.getOrCreate(conf) if Session.active() is None else Session(conf)
        Session._active = self.session
        self.warning()
        self.info(self.describe(self.session))
        if hasattr(self.session, "add_listener"):
            self.session.add_listener(self._on_executor_event)
        self.hide()
        return self.session

    @staticmethod
    def describe(session) -> str:
        pool = getattr(session, "pool", None)
        if pool is None:
            return f"{session!r} -- 1 in-process device: {session.device}"
        return f"{session!r} -- {pool.n} executors: {', '.join(str(d) for d in pool.devices)}"

    def _on_executor_event(self, ev):
        self.warning(f"{ev['event']} ({ev.get('reason')}); DataFrames and models are rebuilt from their "
                     f"sources on next use -- re-run upstream widgets for anything else")
        self.info(self.describe(self.session))

    def onDeleteWidget(self):
        if self.session is not None:
            self.session.stop()
            self.session = None


from ..views import export_views  # noqa: E402

export_views(globals())
