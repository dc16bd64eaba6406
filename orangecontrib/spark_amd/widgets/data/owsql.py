"""Data Frame (SQL) widget: run a query against the session
(reference: widgets/data/spark_sql_dataframe.py:18-100)."""
from orange3_spark_amd.frame.dataframe import DataFrame
from orange3_spark_amd.utils.data_utils import format_sql

from ..base import SharedSession
from ..compat import Setting, Widget


class OWSQLDataFrame(SharedSession, Widget):
    priority = 2
    name = "Data Frame"
    description = "Create a DataFrame from a SQL query"
    icon = "../icons/sql.svg"
    inputs = []
    outputs = [("DataFrame", DataFrame)]
    lastQuery = Setting("")

    def format_query(self, query=None):
        self.lastQuery = format_sql(query if query is not None else self.lastQuery)
        return self.lastQuery

    def execute(self, query=None):
        if query is not None:
            self.lastQuery = query
        if self.session is None:
            self.error("Create a session with the Context widget first")
            return None
        self.error()
        try:
            df = self.session.sql(self.lastQuery)
        except Exception as e:  # noqa: BLE001
            self.error(f"{type(e).__name__}: {e}")
            return None
        self.info(f"{len(df.columns)} columns")
        self.send("DataFrame", df)
        return df


from ..views import export_views  # noqa: E402

export_views(globals())
