"""FillNa widget: ``df.fillna(value, subset)`` (reference widgets/data/spark_fill.py:13-69;
saved values honoured, quirk Q8)."""
from orange3_spark_amd.frame.dataframe import DataFrame

from ...utils.gui_param import coerce
from ...utils.ml_api_utils import get_dataframe_function_info
from ..compat import Setting, Widget


class OWFillNa(Widget):
    priority = 4
    name = "FillNa"
    description = "Replace null / NaN values"
    icon = "../icons/impute.svg"
    inputs = [("DataFrame", DataFrame, "get_input")]
    outputs = [("DataFrame", DataFrame)]
    value = Setting("0")
    subset = Setting("")

    def __init__(self, **kw):
        super().__init__(**kw)
        self.in_df = None
        self.doc = get_dataframe_function_info("fillna")

    def get_input(self, df):
        self.in_df = df

    def apply(self):
        if self.in_df is None:
            return None
        v = coerce(self.value)
        sub = [s.strip() for s in str(self.subset).split(",") if s.strip()] or None
        out = self.in_df.fillna(v, sub)
        self.send("DataFrame", out)
        return out


from ..views import export_views  # noqa: E402

export_views(globals())
