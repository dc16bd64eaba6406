"""to Pandas conversion widget (reference widgets/data/: spark_from_orange.py, spark_from_pandas.py,
spark_to_orange.py, spark_to_pandas.py, pandas_to_orange.py, orange_to_pandas.py; the
duplicate class/display names of the reference are made unique, quirk Q13)."""
import pandas as pd

from orange3_spark_amd.frame.dataframe import DataFrame
from orange3_spark_amd.utils.data_utils import orange_to_pandas, pandas_to_orange

from ..base import SharedSession
from ..compat import Widget


class OWToPandas(SharedSession, Widget):
    priority = 10
    name = "to Pandas"
    description = "Convert DataFrame -> Pandas"
    icon = "../icons/convert.svg"
    inputs = [("DataFrame", DataFrame, "get_input")]
    outputs = [("Pandas", pd.DataFrame)]

    def get_input(self, obj):
        if obj is None:
            self.send("Pandas", None)
            return None
        session = self.session
        if session is None and "session" in "obj.toPandas()":
            from orange3_spark_amd import Session
            session = Session.getOrCreate()
        out = obj.toPandas()
        self.send("Pandas", out)
        return out


_ = (pd, DataFrame, orange_to_pandas, pandas_to_orange)


from ..views import export_views  # noqa: E402

export_views(globals())
