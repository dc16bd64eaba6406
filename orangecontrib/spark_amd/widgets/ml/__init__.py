"""Category "Spark ML (AMD)": reflective estimators/transformers, dataset builder,
model transformer, evaluation, pipeline, tuning, model save/load."""
NAME = "Spark ML (AMD)"
ICON = "../icons/category.svg"
BACKGROUND = "light-orange"
PRIORITY = 101
WIDGET_HELP_PATH = (("{DEVELOP_ROOT}/doc/build/htmlhelp/index.html", None),)
