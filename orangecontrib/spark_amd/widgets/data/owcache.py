"""Cache DataFrame widget: pin the partition in HBM on arrival
(reference widgets/data/spark_df_cache.py:10-40)."""
from orange3_spark_amd.frame.dataframe import DataFrame

from ..compat import Widget


class OWCacheDataFrame(Widget):
    priority = 6
    name = "Cache DataFrame"
    description = "Materialise the DataFrame (and any synthetic lineage) in device memory"
    icon = "../icons/cache.svg"
    inputs = [("DataFrame", DataFrame, "get_input")]
    outputs = [("DataFrame", DataFrame)]

    def get_input(self, df):
        if df is not None:
            df = df.cache()
        self.send("DataFrame", df)


from ..views import export_views  # noqa: E402

export_views(globals())
