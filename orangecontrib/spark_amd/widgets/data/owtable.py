"""Hive Table widget: pick database + table from the catalog
(reference: widgets/data/spark_table.py:13-87; mutable class lists fixed, Q12)."""
from orange3_spark_amd.frame.dataframe import DataFrame

from ..base import SharedSession
from ..compat import Setting, Widget


class OWCatalogTable(SharedSession, Widget):
    priority = 1
    name = "Hive Table"
    description = "Load a DataFrame from a catalog (Hive-style warehouse) table"
    icon = "../icons/table.svg"
    inputs = []
    outputs = [("DataFrame", DataFrame)]
    database = Setting("default")
    table = Setting("")

    def __init__(self, **kw):
        super().__init__(**kw)
        self.databases, self.tables = [], []
        self.refresh()

    def refresh(self):
        if self.session is None:
            return
        self.databases = [r.databaseName for r in self.session.sql("show databases").collect()]
        self.refresh_tables(self.database)

    def refresh_tables(self, db):
        if self.session is not None:
            self.database = db
            self.tables = self.session.tableNames(db)

    def submit(self):
        if self.session is None:
            self.error("Create a session with the Context widget first")
            return None
        name = self.table if self.database in ("", None) else f"{self.database}.{self.table}"
        df = self.session.table(name)
        self.send("DataFrame", df)
        self.hide()
        return df


from ..views import export_views  # noqa: E402

export_views(globals())
