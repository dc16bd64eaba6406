"""Tuning widget (beyond-ref; ml.tuning was listed but unused by the reference,
utils/ml_api_utils.py:76-78): CrossValidator / TrainValidationSplit over a grid given as
``{param: [values...]}`` strings, using the GUI coercion rules."""
from orange3_spark_amd.frame.dataframe import DataFrame
from orange3_spark_amd.ml.base import Evaluator, Model, Params
from orange3_spark_amd.ml.param import ParamGridBuilder
from orange3_spark_amd.ml.tuning import CrossValidator, TrainValidationSplit

from ...utils.gui_param import coerce
from ..compat import Setting, Widget


class OWTuning(Widget):
    priority = 12
    name = "Tuning"
    description = "Cross-validate a stage over a parameter grid"
    icon = "../icons/tuning.svg"
    inputs = [("Stage", Params, "set_stage"), ("Evaluator", Evaluator, "set_evaluator"),
              ("DataFrame", DataFrame, "set_data")]
    outputs = [("Model", Model)]
    method = Setting("CrossValidator")
    numFolds = Setting("3")
    trainRatio = Setting("0.75")
    grid = Setting({})

    def __init__(self, **kw):
        super().__init__(**kw)
        self.stage = self.evaluator = self.in_df = None
        self.metrics = []

    def set_stage(self, s):
        self.stage = s

    def set_evaluator(self, e):
        self.evaluator = e

    def set_data(self, df):
        self.in_df = df

    def apply(self):
        gb = ParamGridBuilder()
        for name, vals in self.grid.items():
            v = coerce(vals) if isinstance(vals, str) else vals
            gb.addGrid(self.stage.getParam(name), v if isinstance(v, list) else [v])
        maps = gb.build()
        if self.method == "CrossValidator":
            t = CrossValidator(estimator=self.stage, estimatorParamMaps=maps, evaluator=self.evaluator,
                               numFolds=int(coerce(self.numFolds)))
        else:
            t = TrainValidationSplit(estimator=self.stage, estimatorParamMaps=maps, evaluator=self.evaluator,
                                     trainRatio=float(coerce(self.trainRatio)))
        m = t.fit(self.in_df)
        self.metrics = getattr(m, "avgMetrics", None) or getattr(m, "validationMetrics", [])
        self.send("Model", m)
        return m


from ..views import export_views  # noqa: E402

export_views(globals())
