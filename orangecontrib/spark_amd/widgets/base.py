"""Shared widget bases: the process-global session and the reflective ML widgets.

* :class:`SharedSession` -- every widget sees the session the Context widget created
  (reference SharedSparkContext, orangecontrib/spark/base/shared_spark_context.py:9-27:
  class attributes ``sc``/``hc``; here ``session`` plus ``sc``/``hc`` aliases).
* :class:`OWTransformerBase` -- reflective "pick any Transformer of <module>" widget
  (reference OWSparkTransformer, base/spark_ml_transformer.py:16-139).
* :class:`OWEstimatorBase` -- same but calls ``fit`` and outputs a Model
  (reference OWSparkEstimator, base/spark_ml_estimator.py:10-25).

Fixes of reference quirks: ``None`` GUI values mean "use the default" (Q10), saved values
are honoured, a failing apply reports through ``self.error`` instead of raising (Q14 runs
fit in a worker thread in the Qt view; headless calls are synchronous).  Beyond the
reference, both widgets also output the configured (unfitted) stage on "Stage" so it can
be wired into the Pipeline widget.
"""
from __future__ import annotations

import traceback
from collections import OrderedDict

from orange3_spark_amd.frame.dataframe import DataFrame
from orange3_spark_amd.ml.base import Model, Params

from ..utils.gui_param import GuiParam
from ..utils.ml_api_utils import get_estimators, get_object_info, get_transformers
from .compat import Default, Dynamic, Setting, Widget


class SharedSession:
    """Mixin giving every widget the process-global Session (the 'shared context')."""

    _session = None

    @property
    def session(self):
        from orange3_spark_amd import Session
        return SharedSession._session if SharedSession._session is not None else Session.active()

    @session.setter
    def session(self, val):
        SharedSession._session = val

    # reference-compatible aliases (sc = SparkContext, hc = HiveContext)
    @property
    def sc(self):
        s = self.session
        return s.sparkContext if s is not None else None

    @sc.setter
    def sc(self, val):
        self.session = getattr(val, "session", val)

    hc = session


class OWTransformerBase(SharedSession, Widget):
    name = "Transformer"
    description = "A Transformer of the ML API"
    icon = "icons/transformer.svg"
    inputs = [("DataFrame", DataFrame, "get_input", Default)]
    outputs = [("DataFrame", DataFrame, Dynamic), ("Stage", Params, Dynamic)]

    module = None
    get_modules = staticmethod(get_transformers)
    saved_gui_params = Setting(OrderedDict())
    var_cache_check = Setting(False)

    def __init__(self, **kw):
        super().__init__(**kw)
        self.in_df = None
        self.out_df = None
        self.gui_parameters: "OrderedDict[str, GuiParam]" = OrderedDict()
        self.module_methods = self.get_modules(None, self.module)
        self.method_names = sorted(self.module_methods.keys())
        default = self.saved_gui_params.get("method", None)
        self.gui_parameters["method"] = GuiParam(list_values=self.method_names or [""], default_value=default,
                                                 callback_func=self.refresh_method)
        self.method = None
        self.method_parameters = OrderedDict()
        self.method_info = ""
        if self.method_names:
            self.refresh_method(self.gui_parameters["method"].get_value())

    # -- method selection / parameter editors --------------------------------------
    def refresh_method(self, text):
        self.method = self.module_methods[text]
        _, _, self.method_parameters, self.method_info = get_object_info(self.method)
        for k in list(self.gui_parameters):
            if k != "method":
                del self.gui_parameters[k]
        for k, v in self.method_parameters.items():
            default_value, doc = v[1], v[-1] if len(v) > 2 else ""
            list_values = None
            if k.endswith("Col") and self.in_df is not None:
                list_values = [str(default_value)] + list(self.in_df.columns)
            saved = self.saved_gui_params.get(k) if self.saved_gui_params.get("method") == text else None
            value = saved if saved is not None else str(default_value)
            if list_values is not None and value not in list_values:
                list_values.append(value)
            self.gui_parameters[k] = GuiParam(label=k, default_value=value, list_values=list_values,
                                              place_holder_text=doc, doc_text=doc)

    def select_method(self, name: str):
        self.gui_parameters["method"].set_value(name)
        return self

    def set_param(self, name: str, value) -> "OWTransformerBase":
        self.gui_parameters[name].set_value(value)
        return self

    def get_input(self, obj):
        self.in_df = obj
        self.refresh_method(self.gui_parameters["method"].get_value())

    def build_param_map(self, method_instance) -> dict:
        from orange3_spark_amd.ml.param import Param
        pm = {}
        for k in self.method_parameters:
            value = self.gui_parameters[k].get_usable_value()
            if value is None:                 # Q10: blank / None -> keep the default
                continue
            pm[Param(method_instance, k, "")] = value
        return pm

    def configured_stage(self):
        inst = self.method()
        for p, v in self.build_param_map(inst).items():
            inst.set(p.name, v)
        return inst

    def update_saved_gui_parameters(self):
        for k, p in self.gui_parameters.items():
            self.saved_gui_params[k] = p.get_value()

    def apply(self):
        self.error()
        try:
            inst = self.method()
            pm = self.build_param_map(inst)
            self.send("Stage", self.configured_stage())
            if self.in_df is None:
                self.update_saved_gui_parameters()
                return None
            self.out_df = inst.transform(self.in_df, params=pm)
            if self.var_cache_check:
                self.out_df = self.out_df.cache()
            self.send("DataFrame", self.out_df)
            self.update_saved_gui_parameters()
            self.hide()
            return self.out_df
        except Exception as e:  # noqa: BLE001
            self.error(f"{type(e).__name__}: {e}")
            self.last_traceback = traceback.format_exc()
            return None


class OWEstimatorBase(OWTransformerBase):
    name = "Estimator"
    description = "An Estimator of the ML API"
    icon = "icons/estimator.svg"
    outputs = [("Model", Model, Dynamic), ("Stage", Params, Dynamic)]
    get_modules = staticmethod(get_estimators)

    def apply(self):
        self.error()
        try:
            inst = self.method()
            pm = self.build_param_map(inst)
            self.send("Stage", self.configured_stage())
            if self.in_df is None:
                self.update_saved_gui_parameters()
                return None
            self.out_model = inst.fit(self.in_df, params=pm)
            self.send("Model", self.out_model)
            self.update_saved_gui_parameters()
            self.hide()
            return self.out_model
        except Exception as e:  # noqa: BLE001
            self.error(f"{type(e).__name__}: {e}")
            self.last_traceback = traceback.format_exc()
            return None
