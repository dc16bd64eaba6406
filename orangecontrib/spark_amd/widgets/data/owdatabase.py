"""Database widget (reference "ODBC", widgets/data/odbc_table.py:29-216): run SQL on a
DB-API connection and output an Orange Table, its Domain and a pandas DataFrame.
pyodbc is not available here, so the driver is pluggable: ``sqlite3`` (stdlib) by default,
pyodbc when importable (quirk Q7 fixed: the query is a persisted setting and is used)."""
import pandas as pd

from orange3_spark_amd.utils.data_utils import format_sql, pandas_to_orange

from ..compat import Setting, Widget


class OWDatabase(Widget):
    priority = 3
    name = "Database"
    description = "Query a DB-API database (sqlite3 / ODBC) into Orange and pandas tables"
    icon = "../icons/database.svg"
    inputs = []
    outputs = [("Data", object), ("Feature Definitions", object), ("Pandas", pd.DataFrame)]
    driver = Setting("sqlite3")
    connectString = Setting(":memory:")
    lastQuery = Setting("")

    def __init__(self, **kw):
        super().__init__(**kw)
        self.conn = None

    @staticmethod
    def data_sources():
        try:
            import pyodbc
            return sorted(pyodbc.dataSources())
        except Exception:  # noqa: BLE001
            return []

    def connect(self):
        if self.driver == "pyodbc":
            import pyodbc
            self.conn = pyodbc.connect(self.connectString)
        else:
            import sqlite3
            self.conn = sqlite3.connect(self.connectString)
        return self.conn

    def format_query(self):
        self.lastQuery = format_sql(self.lastQuery)
        return self.lastQuery

    def execute_query(self, query=None):
        if query is not None:
            self.lastQuery = query
        if self.conn is None:
            self.connect()
        pdf = pd.read_sql_query(self.lastQuery, self.conn)
        table = pandas_to_orange(pdf.copy())
        self.send("Data", table)
        self.send("Feature Definitions", table.domain)
        self.send("Pandas", pdf)
        self.info(f"{len(pdf)} rows")
        return pdf


from ..views import export_views  # noqa: E402

export_views(globals())
