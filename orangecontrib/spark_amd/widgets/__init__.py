"""Widget packages of the add-on (categories: data, ml)."""
WIDGET_HELP_PATH = (
    ("{DEVELOP_ROOT}/doc/build/htmlhelp/index.html", None),
)
