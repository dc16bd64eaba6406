"""Catalog: the "Hive" replacement -- databases and tables in a parquet warehouse.

The reference's Hive Table widget lists databases with ``hc.sql("show databases")``
and tables with ``hc.tableNames(db)``, then loads ``hc.table(db + '.' + table)``
(orangecontrib/spark/widgets/data/spark_table.py:40-41,59-70,75-83).  Layout follows
Hive's warehouse convention: tables of ``default`` live in ``<warehouse>/<table>/``,
other databases in ``<warehouse>/<db>.db/<table>/``; each table is a Spark-style
parquet directory (one part file per writing rank).  Temp views live in memory.
"""
from __future__ import annotations

import os
import shutil

from .frame.dataframe import DataFrame


class Database:
    def __init__(self, name, description="", locationUri=""):
        self.name, self.description, self.locationUri = name, description, locationUri

    def __repr__(self):
        return f"Database(name={self.name!r}, locationUri={self.locationUri!r})"


class Table:
    def __init__(self, name, database, isTemporary=False, tableType="MANAGED"):
        self.name, self.database, self.isTemporary, self.tableType = name, database, isTemporary, tableType

    def __repr__(self):
        return f"Table(name={self.name!r}, database={self.database!r}, isTemporary={self.isTemporary})"


class Catalog:
    def __init__(self, session):
        self.session = session
        self._temp: dict[str, DataFrame] = {}
        self._cached: dict[str, DataFrame] = {}
        self._current = "default"

    # ------------------------------------------------------------------ paths
    @property
    def warehouse(self) -> str:
        return os.path.abspath(self.session.conf.warehouse())

    def _db_path(self, db: str) -> str:
        return self.warehouse if db == "default" else os.path.join(self.warehouse, f"{db}.db")

    def _split(self, name: str) -> tuple[str, str]:
        if "." in name:
            db, t = name.split(".", 1)
            return db, t
        return self._current, name

    def _table_path(self, name: str) -> str:
        db, t = self._split(name)
        return os.path.join(self._db_path(db), t)

    # ------------------------------------------------------------------ databases
    def currentDatabase(self) -> str:
        return self._current

    def setCurrentDatabase(self, db: str) -> None:
        if db not in self.databaseNames():
            raise ValueError(f"Database '{db}' not found")
        self._current = db

    def databaseNames(self) -> list[str]:
        names = {"default"}
        if os.path.isdir(self.warehouse):
            for e in os.listdir(self.warehouse):
                if e.endswith(".db") and os.path.isdir(os.path.join(self.warehouse, e)):
                    names.add(e[:-3])
        return sorted(names)

    def listDatabases(self) -> list[Database]:
        return [Database(n, "", self._db_path(n)) for n in self.databaseNames()]

    def createDatabase(self, db: str, ifNotExists: bool = True) -> None:
        p = self._db_path(db)
        if os.path.isdir(p) and db != "default" and not ifNotExists:
            raise FileExistsError(f"Database '{db}' already exists")
        if self.session.comm.rank == 0:
            os.makedirs(p, exist_ok=True)
        self.session.comm.barrier()

    def dropDatabase(self, db: str, cascade: bool = False) -> None:
        if db == "default":
            raise ValueError("cannot drop default database")
        if self.session.comm.rank == 0 and os.path.isdir(self._db_path(db)):
            shutil.rmtree(self._db_path(db))
        self.session.comm.barrier()

    # ------------------------------------------------------------------ tables
    def tableNames(self, dbName: str | None = None) -> list[str]:
        db = dbName or self._current
        p = self._db_path(db)
        names = []
        if os.path.isdir(p):
            for e in sorted(os.listdir(p)):
                full = os.path.join(p, e)
                if os.path.isdir(full) and not e.endswith(".db") and not e.startswith((".", "_")):
                    names.append(e)
        if db == self._current:
            names += sorted(k for k in self._temp if k not in names)
        return names

    def listTables(self, dbName: str | None = None) -> list[Table]:
        db = dbName or self._current
        return [Table(n, None if n in self._temp else db, n in self._temp) for n in self.tableNames(db)]

    def tableExists(self, name: str, dbName: str | None = None) -> bool:
        if dbName:
            name = f"{dbName}.{name}"
        return name in self._temp or os.path.isdir(self._table_path(name))

    def table(self, name: str) -> DataFrame:
        if name.startswith("global_temp."):
            from .frame.extras import _GLOBAL_TEMP
            if name[12:] in _GLOBAL_TEMP:
                return _GLOBAL_TEMP[name[12:]]
            raise KeyError(f"Table or view not found: {name}")
        if name in self._temp:
            return self._temp[name]
        if name in self._cached:
            return self._cached[name]
        p = self._table_path(name)
        if not os.path.isdir(p):
            raise KeyError(f"Table or view not found: {name}")
        from .io import read_parquet
        return read_parquet(self.session, p)

    def saveAsTable(self, df: DataFrame, name: str, mode: str = "error") -> None:
        from .io import write_parquet
        db, t = self._split(name)
        if db != "default" and db not in self.databaseNames():
            self.createDatabase(db)
        p = self._table_path(name)
        if mode == "append" and os.path.isdir(p):
            df = self.table(name).union(df.select(*self.table(name).columns))
            mode = "overwrite"
        write_parquet(df, p, mode)

    def dropTable(self, name: str) -> None:
        p = self._table_path(name)
        if self.session.comm.rank == 0 and os.path.isdir(p):
            shutil.rmtree(p)
        self.session.comm.barrier()

    def registerTempView(self, name: str, df: DataFrame) -> None:
        self._temp[name] = df

    def dropGlobalTempView(self, name: str) -> bool:
        from .frame.extras import _GLOBAL_TEMP
        return _GLOBAL_TEMP.pop(name, None) is not None

    def dropTempView(self, name: str) -> bool:
        return self._temp.pop(name, None) is not None

    def cacheTable(self, name: str) -> None:
        """Materialise the table in device memory; later ``table(name)`` calls reuse it."""
        df = self.table(name).cache()
        self._cached[name] = df

    def isCached(self, name: str) -> bool:
        return name in self._cached or (name in self._temp and getattr(self._temp[name], "is_cached", False))

    def uncacheTable(self, name: str) -> None:
        self._cached.pop(name, None)
        view = self._temp.get(name)
        if view is not None and hasattr(view, "unpersist"):
            view.unpersist()

    def clearCache(self) -> None:
        self._cached.clear()

    def refreshTable(self, name: str) -> None:
        """Drop any cached copy so the next read sees the files on disk."""
        self._cached.pop(name, None)

    def databaseExists(self, dbName: str) -> bool:
        return dbName in self.databaseNames()

    def getDatabase(self, dbName: str) -> Database:
        if not self.databaseExists(dbName):
            raise KeyError(f"Database not found: {dbName}")
        return Database(dbName, locationUri=self._db_path(dbName))

    def getTable(self, tableName: str) -> Table:
        if tableName in self._temp:
            return Table(tableName, None, True)
        if not self.tableExists(tableName):
            raise KeyError(f"Table or view not found: {tableName}")
        db, t = self._split(tableName)
        return Table(t, db, False)

    def listColumns(self, tableName: str, dbName: str | None = None) -> list:
        """Column(name, description, dataType, nullable, isPartition, isBucket) entries."""
        from collections import namedtuple
        Column = namedtuple("Column", "name description dataType nullable isPartition isBucket")
        df = self.table(f"{dbName}.{tableName}" if dbName else tableName)
        return [Column(f.name, None, f.dataType.simpleString(), True, False, False) for f in df.schema.fields]

    def listFunctions(self, dbName: str | None = None) -> list:
        """Built-in SQL functions (sql/functions.py) and registered UDFs (spark.udf)."""
        import inspect
        from collections import namedtuple
        from .sql import functions as F
        from .sql import udf as U
        Function = namedtuple("Function", "name description className isTemporary")
        names = sorted(n for n, v in vars(F).items() if callable(v) and not n.startswith("_")
                       and not inspect.isclass(v) and getattr(v, "__module__", "").startswith("orange3_spark_amd"))
        out = [Function(n, None, "builtin", False) for n in names]
        out += [Function(n, None, "python_udf", True) for n in sorted(U._REGISTRY)]
        return out

    def functionExists(self, functionName: str, dbName: str | None = None) -> bool:
        return any(f.name.lower() == functionName.lower() for f in self.listFunctions())

    def createTable(self, tableName: str, path: str | None = None, source: str | None = None, schema=None,
                    **options):
        """Register files at ``path`` (parquet / csv / json) as a catalog table, or create an
        empty table from ``schema``; returns it as a DataFrame."""
        if path is not None:
            df = self.session.read.load(path, format=source or "parquet", **options)
        else:
            names = [f.name for f in getattr(schema, "fields", [])]
            import pandas as pd
            df = self.session.createDataFrame(pd.DataFrame({n: pd.Series([], dtype=float) for n in names}))
        self.saveAsTable(df, tableName, "overwrite")
        return self.table(tableName)

    createExternalTable = createTable
