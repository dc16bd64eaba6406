"""Sample widget: ``df.sample(withReplacement, fraction, seed)``
(reference widgets/data/spark_sample.py:13-72; defaults False/0.5/1, saved values honoured)."""
from orange3_spark_amd.frame.dataframe import DataFrame

from ...utils.gui_param import coerce
from ..compat import Setting, Widget


class OWSample(Widget):
    priority = 5
    name = "Sample"
    description = "Bernoulli/Poisson row sample (identical on any GPU count)"
    icon = "../icons/sample.svg"
    inputs = [("DataFrame", DataFrame, "get_input")]
    outputs = [("DataFrame", DataFrame)]
    withReplacement = Setting("False")
    fraction = Setting("0.5")
    seed = Setting("1")

    def __init__(self, **kw):
        super().__init__(**kw)
        self.in_df = None

    def get_input(self, df):
        self.in_df = df

    def apply(self):
        if self.in_df is None:
            return None
        out = self.in_df.sample(bool(coerce(self.withReplacement)), float(coerce(self.fraction)),
                                int(coerce(self.seed)))
        self.send("DataFrame", out)
        return out


from ..views import export_views  # noqa: E402

export_views(globals())
