"""Pipeline widget (beyond-ref): chain configured stages (from the reflective widgets'
"Stage" outputs, in link order) into ``Pipeline(stages).fit(df)``."""
from collections import OrderedDict

from orange3_spark_amd.frame.dataframe import DataFrame
from orange3_spark_amd.ml.base import Model, Params, Pipeline

from ..compat import Multiple, Widget


class OWPipeline(Widget):
    priority = 10
    name = "Pipeline"
    description = "Fit a Pipeline of Estimator/Transformer stages"
    icon = "../icons/pipeline.svg"
    inputs = [("Stage", Params, "add_stage", Multiple), ("DataFrame", DataFrame, "set_data")]
    outputs = [("Model", Model), ("Pipeline", Pipeline)]

    def __init__(self, **kw):
        super().__init__(**kw)
        self.stages = OrderedDict()
        self.in_df = None

    def add_stage(self, stage, key=None):
        key = key if key is not None else len(self.stages)
        if stage is None:
            self.stages.pop(key, None)
        else:
            self.stages[key] = stage

    def set_data(self, df):
        self.in_df = df

    def apply(self):
        pipe = Pipeline(stages=list(self.stages.values()))
        self.send("Pipeline", pipe)
        if self.in_df is None:
            return pipe
        self.error()
        try:
            model = pipe.fit(self.in_df)
        except Exception as e:  # noqa: BLE001
            self.error(f"{type(e).__name__}: {e}")
            return None
        self.send("Model", model)
        return model


from ..views import export_views  # noqa: E402

export_views(globals())
