from .dataframe import DataFrame, GroupedData, Row  # noqa: F401
from . import expr as functions  # noqa: F401
from . import types  # noqa: F401
