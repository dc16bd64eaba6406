"""SQL surface: parser/engine (``session.sql``), ``functions`` and ``Window``."""
from .window import Window, WindowSpec  # noqa: F401
