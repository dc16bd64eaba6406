"""Cache DataFrame widget: pin the partition on arrival
(reference widgets/data/spark_df_cache.py:10-40, ``in_df.cache()``).

``storageLevel`` (beyond-ref): ``MEMORY_ONLY`` (default: HBM; rows of a synthetic table
beyond the budget are recomputed from lineage), ``MEMORY_AND_DISK`` (vector rows beyond the
HBM budget kept in pinned host memory and streamed through every pass) or ``DISK_ONLY``."""
from orange3_spark_amd.frame.dataframe import DataFrame, StorageLevel

from ..compat import Setting, Widget

LEVELS = ("MEMORY_ONLY", "MEMORY_AND_DISK", "DISK_ONLY")


class OWCacheDataFrame(Widget):
    priority = 6
    name = "Cache DataFrame"
    description = "Materialise the DataFrame (and any synthetic lineage) in device memory"
    icon = "../icons/cache.svg"
    inputs = [("DataFrame", DataFrame, "get_input")]
    outputs = [("DataFrame", DataFrame)]
    storageLevel = Setting("MEMORY_ONLY")

    def get_input(self, df):
        self.error()
        if df is not None:
            lvl = str(self.storageLevel or "MEMORY_ONLY").strip().upper()
            if lvl not in LEVELS:
                self.error(f"storageLevel must be one of {', '.join(LEVELS)}")
                lvl = StorageLevel.MEMORY_ONLY
            df = df.cache() if lvl == StorageLevel.MEMORY_ONLY else df.persist(lvl)
            self.info(f"cached ({lvl})")
        self.send("DataFrame", df)


from ..views import export_views  # noqa: E402

export_views(globals())
