"""Category "Spark Data (AMD)": session, sources, DataFrame operations, conversions."""
NAME = "Spark Data (AMD)"
ICON = "../icons/category.svg"
BACKGROUND = "white"
PRIORITY = 100
WIDGET_HELP_PATH = (("{DEVELOP_ROOT}/doc/build/htmlhelp/index.html", None),)
