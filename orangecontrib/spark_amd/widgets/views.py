"""Qt views of the headless widgets, generated when Orange3 is importable.

The reference's widgets are Qt ``OWWidget`` subclasses whose logic lives inside the Qt
class (e.g. reference base/spark_ml_transformer.py:16-139 builds its combo boxes and runs
``fit`` from the Apply button; widgets/data/spark_table.py:13-87 fills two list views).
Here every widget's logic is a headless :class:`compat.Widget` (fully tested without Qt)
and this module wraps each one in a thin Qt shell:

* old-style ``inputs``/``outputs`` tuples become ``Inputs``/``Outputs`` signal classes whose
  handlers forward to the headless handler, and the headless ``send`` is bridged to
  ``self.Outputs.<channel>.send``;
* every ``compat.Setting`` becomes an ``Orange.widgets.settings.Setting`` (workflow
  persistence) and gets an editor (check box for bools, line edit for scalars);
* reflective ML widgets get one editor per :class:`GuiParam` -- a combo box when it has
  ``list_values``, a line edit otherwise -- rebuilt when the method combo changes;
* the widget's action (``apply``/``commit``/``submit``/``create_context``/``execute``)
  runs from an Apply button, on a worker thread when Orange's ``ConcurrentWidgetMixin``
  exists (reference quirk Q14: ``fit`` froze the GUI), with the fit's progress
  (runtime/progress.py) reported to the task's progress bar and Cancel honoured at the
  next iteration; outputs AND messages produced on the worker are queued and delivered on
  the GUI thread when the task finishes (Qt widgets are touched from the GUI thread only);
* ``info``/``warning``/``error`` of the headless widget show up as the view's
  ``information``/``warning``/``error`` messages (``OWBaseWidget.info`` is the StateInfo
  summary, not a message method) and a ``table()`` (Evaluation) or the output DataFrame
  preview fills the main area.

Each ``ow*.py`` module calls :func:`export_views` at import time; with Orange absent that
is a no-op, with Orange present it adds ``<Class>View`` next to the headless class with
``__module__`` set to that module, which is where Orange's widget discovery looks.
"""
from __future__ import annotations

import copy
import html
import re
import threading

from .compat import HAVE_ORANGE, Multiple, Setting, Widget

_ACTIONS = ("apply", "commit", "submit", "create_context", "execute")


def _ident(channel: str) -> str:
    s = re.sub(r"\W+", "_", channel).strip("_").lower()
    return s if s and not s[0].isdigit() else "ch_" + s


class _Bridge:
    """Stands in as the headless widget's signal manager: forwards ``send`` and the
    ``info``/``warning``/``error`` messages to the Qt widget when called on the GUI thread,
    and queues them (in order) while the action runs on a worker thread -- Qt widgets may
    only be touched from the GUI thread; :meth:`flush` runs there when the task ends."""

    def __init__(self, view):
        self.view = view
        self.pending = []
        self._lock = threading.Lock()

    @staticmethod
    def _on_gui_thread() -> bool:
        return threading.current_thread() is threading.main_thread()

    def send(self, _src, channel, value):
        if self._on_gui_thread():
            self.view._emit(channel, value)
        else:
            with self._lock:
                self.pending.append(("send", channel, value))

    def message(self, level, text):
        if self._on_gui_thread():
            self.view._show_message(level, text)
        else:
            with self._lock:
                self.pending.append(("message", level, text))

    def flush(self):
        with self._lock:
            pending, self.pending = self.pending, []
        for kind, a, b in pending:
            if kind == "send":
                self.view._emit(a, b)
            else:
                self.view._show_message(a, b)


# headless message level -> OWBaseWidget method (``OWBaseWidget.info`` is the widget's
# StateInfo summary object, not a message method)
_MESSAGE_METHOD = {"info": "information", "warning": "warning", "error": "error"}


def _settings_of(core_cls):
    out = {}
    for k in dir(core_cls):
        v = getattr(core_cls, k, None)
        if isinstance(v, Setting):
            out[k] = v
    return out


def qt_view(core_cls, orange=None):
    """Build the Qt ``OWWidget`` class for headless widget ``core_cls``.

    ``orange`` is a namespace with ``widget``, ``settings``, ``gui`` and ``qt`` (the
    AnyQt.QtWidgets module; optionally ``qtgui`` / ``qtcore`` for the script editor's
    highlighter and key handling); by default the real Orange/AnyQt modules are imported.
    """
    if orange is None:
        from types import SimpleNamespace

        from AnyQt import QtCore, QtGui, QtWidgets
        from Orange.widgets import gui, settings, widget
        try:
            from Orange.widgets.utils.concurrent import ConcurrentWidgetMixin
        except ImportError:  # older Orange: run the action on the GUI thread
            ConcurrentWidgetMixin = None
        orange = SimpleNamespace(widget=widget, settings=settings, gui=gui, qt=QtWidgets,
                                 qtgui=QtGui, qtcore=QtCore, concurrent=ConcurrentWidgetMixin)
    W, S, Qt = orange.widget, orange.settings, orange.qt
    Mixin = getattr(orange, "concurrent", None)

    class Inputs:
        pass

    class Outputs:
        pass

    ns = {}
    out_attr = {}
    for spec in core_cls.outputs:
        name, typ = spec[0], spec[1]
        setattr(Outputs, _ident(name), W.Output(name, typ))
        out_attr[name] = _ident(name)
    for spec in core_cls.inputs:
        name, typ, handler = spec[0], spec[1], spec[2]
        flags = spec[3] if len(spec) > 3 else 0
        inp = W.Input(name, typ, multiple=bool(flags & Multiple))
        setattr(Inputs, _ident(name), inp)

        def forward(self, value, *_id, _h=handler):
            getattr(self.core, _h)(value)
            self._refresh_editors()
            self._show_result()
        forward.__name__ = "set_" + _ident(name)
        ns[forward.__name__] = inp(forward)

    core_settings = _settings_of(core_cls)
    for k, st in core_settings.items():
        # a copy: the Qt class's setting must not share the headless class's mutable
        # default (a view instance that edits it in place would change every later
        # headless widget's default)
        ns[k] = S.Setting(copy.deepcopy(st.default))
    has_table = callable(getattr(core_cls, "table", None))      # Evaluation's Metric|Value table
    action = next((a for a in _ACTIONS if callable(getattr(core_cls, a, None))), None)

    def __init__(self, *a, **kw):
        W.OWWidget.__init__(self, *a, **kw)
        if Mixin is not None:
            Mixin.__init__(self)
        self.core = core_cls(**{k: getattr(self, k) for k in core_settings})
        self.bridge = _Bridge(self)
        self.core.signal_manager = self.bridge
        for level in ("info", "warning", "error"):
            setattr(self.core, level, self._message_forwarder(level))
        self._param_box = None
        self._build_controls()

    def _message_forwarder(self, level):
        def fwd(text=None):
            self.core.messages[level] = text          # headless state: any thread
            self.bridge.message(level, text)          # the Qt message: GUI thread only
        return fwd

    def _show_message(self, level, text):
        shown = getattr(self, _MESSAGE_METHOD[level], None)
        if callable(shown):
            shown(text) if text else shown()

    def _emit(self, channel, value):
        getattr(self.Outputs, out_attr[channel]).send(value)
        self._show_result()

    # -- controls ---------------------------------------------------------------------
    def _build_controls(self):
        from .custom_views import BUILDERS
        covered = set()
        self._custom_refresh = None
        builder = BUILDERS.get(core_cls.__name__)
        if builder is not None:                # hand-written list / editor controls
            covered, self._custom_refresh = builder(self, orange)
        box = orange.gui.widgetBox(self.controlArea, "Settings")
        for k, st in core_settings.items():
            if k in covered:
                continue
            if isinstance(st.default, bool):
                orange.gui.checkBox(box, self, k, k, callback=lambda k=k: self._sync(k))
            elif st.default is None or isinstance(st.default, (str, int, float)):
                orange.gui.lineEdit(box, self, k, label=k, callback=lambda k=k: self._sync(k))
        if hasattr(self.core, "gui_parameters"):
            self._param_box = orange.gui.widgetBox(self.controlArea, "Parameters")
            self._refresh_editors()
        if action is not None:
            orange.gui.button(self.controlArea, self, action.replace("_", " ").title(), callback=self.run_action)
        if core_cls.want_main_area or has_table:
            self.result_view = Qt.QTextBrowser()
            self.mainArea.layout().addWidget(self.result_view)
        else:
            self.result_view = None

    def _sync(self, k):
        setattr(self.core, k, getattr(self, k))

    def _refresh_editors(self):
        if self._custom_refresh is not None:
            self._custom_refresh()
        if self._param_box is None:
            return
        lay = self._param_box.layout()
        while lay.count():
            item = lay.takeAt(0)
            if item.widget() is not None:
                item.widget().deleteLater()
        for name, gp in self.core.gui_parameters.items():
            lay.addWidget(Qt.QLabel(gp.label or name))
            if gp.list_values:
                ed = Qt.QComboBox()
                ed.addItems([str(v) for v in gp.list_values])
                ed.setCurrentText(str(gp.get_value()))
                ed.currentTextChanged.connect(lambda text, n=name: self._param_changed(n, text))
            else:
                ed = Qt.QLineEdit(str(gp.get_value()))
                if gp.place_holder_text:
                    ed.setPlaceholderText(str(gp.place_holder_text))
                ed.textChanged.connect(lambda text, n=name: self._param_changed(n, text))
            if gp.doc_text:
                ed.setToolTip(str(gp.doc_text))
            lay.addWidget(ed)

    def _param_changed(self, name, text):
        self.core.gui_parameters[name].set_value(text)
        if name == "method":
            self._refresh_editors()

    # -- action ----------------------------------------------------------------------
    def run_action(self):
        for k in core_settings:
            self._sync(k)
        fn = getattr(self.core, action)
        if Mixin is not None:
            def task(state):
                # the fit's per-iteration / per-tree progress goes to the task state (Orange
                # delivers it to the GUI thread's progress bar); Cancel stops the fit at its
                # next iteration (runtime/progress.py)
                from orange3_spark_amd.runtime.progress import progress_scope, report
                with progress_scope(getattr(state, "set_progress_value", None),
                                    getattr(state, "is_interruption_requested", None)):
                    out = fn()
                    report(1.0)
                    return out
            self.start(task)
        else:
            fn()
            self.on_done(None)

    def on_done(self, _result):
        self.bridge.flush()
        for k in core_settings:               # the action may update settings (saved params)
            setattr(self, k, getattr(self.core, k))
        if self._custom_refresh is not None:
            self._custom_refresh()
        self._show_result()

    def on_exception(self, ex):
        self.bridge.flush()
        self.core.error(f"{type(ex).__name__}: {ex}")

    def _show_result(self):
        if self.result_view is None:
            return
        rows = None
        if has_table:
            rows = self.core.table()
        else:
            df = getattr(self.core, "out_df", None)
            df = getattr(self.core, "in_df", None) if df is None else df
            if df is not None:
                pdf = df.limit(20).toPandas()
                rows = [tuple(pdf.columns)] + [tuple(r) for r in pdf.itertuples(index=False)]
        if rows:
            head, *body = rows
            cells = "".join(f"<th>{html.escape(str(h))}</th>" for h in head)
            trs = "".join("<tr>" + "".join(f"<td>{html.escape(str(v))}</td>" for v in r) + "</tr>" for r in body)
            self.result_view.setHtml(f"<table border=1><tr>{cells}</tr>{trs}</table>")

    def onDeleteWidget(self):
        self.core.onDeleteWidget()
        if Mixin is not None:
            self.shutdown()
        W.OWWidget.onDeleteWidget(self)

    ns.update(dict(
        name=core_cls.name, description=core_cls.description, icon=core_cls.icon, priority=core_cls.priority,
        want_main_area=bool(core_cls.want_main_area or has_table),
        resizing_enabled=core_cls.resizing_enabled, Inputs=Inputs, Outputs=Outputs, core_class=core_cls,
        __init__=__init__, _message_forwarder=_message_forwarder, _show_message=_show_message, _emit=_emit,
        _build_controls=_build_controls,
        _sync=_sync, _refresh_editors=_refresh_editors, _param_changed=_param_changed, run_action=run_action,
        on_done=on_done, on_exception=on_exception, _show_result=_show_result, onDeleteWidget=onDeleteWidget,
        __module__=core_cls.__module__, __qualname__=core_cls.__name__ + "View"))
    bases = (W.OWWidget,) if Mixin is None else (W.OWWidget, Mixin)
    return type(core_cls.__name__ + "View", bases, ns)


def export_views(module_globals: dict, orange=None) -> list:
    """Add a Qt view next to every headless widget class defined in a widget module."""
    if orange is None and not HAVE_ORANGE:
        return []
    made = []
    mod = module_globals.get("__name__")
    for name, obj in list(module_globals.items()):
        if isinstance(obj, type) and issubclass(obj, Widget) and obj.__module__ == mod \
                and not name.startswith("_") and getattr(obj, "name", None):
            view = qt_view(obj, orange)
            module_globals[name + "View"] = view
            made.append(view)
    return made
