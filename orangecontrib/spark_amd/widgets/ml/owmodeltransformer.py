"""Model Transformer: ``model.transform(df)`` once both inputs are present
(reference widgets/ml/spark_ml_model.py:11-54)."""
from orange3_spark_amd.frame.dataframe import DataFrame
from orange3_spark_amd.ml.base import Model, Transformer

from ..compat import Widget


class OWModelTransformer(Widget):
    priority = 8
    name = "Model Transformer"
    description = "Apply a fitted model (or any transformer) to a DataFrame"
    icon = "../icons/model.svg"
    inputs = [("DataFrame", DataFrame, "get_input"), ("Model", Transformer, "get_input_model")]
    outputs = [("DataFrame", DataFrame)]

    def __init__(self, **kw):
        super().__init__(**kw)
        self.in_df = self.in_model = self.out_df = None

    def get_input(self, df):
        self.in_df = df
        self.transform()

    def get_input_model(self, model):
        self.in_model = model
        self.transform()

    def transform(self):
        if self.in_df is not None and self.in_model is not None:
            self.error()
            try:
                self.out_df = self.in_model.transform(self.in_df)
            except Exception as e:  # noqa: BLE001
                self.error(f"{type(e).__name__}: {e}")
                return None
            self.send("DataFrame", self.out_df)
            return self.out_df
        return None


_ = Model


from ..views import export_views  # noqa: E402

export_views(globals())
