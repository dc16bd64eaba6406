"""SQL surface: parser/engine (``session.sql``), ``functions`` and ``Window``."""
from .window import Window, WindowSpec  # noqa: F401
from .functions import grouping, grouping_id  # noqa: F401,E402
from ..frame.extras import Observation  # noqa: F401,E402
