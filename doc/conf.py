# Sphinx configuration for the generated reference (doc/*.md, written by tools/make_docs.py).
# The reference add-on shipped only a template conf.py (doc/conf.py there); these pages are
# the widget help its WIDGET_HELP_PATH points at.  Build: sphinx-build -b html doc doc/build/htmlhelp
project = "Orange3-Spark-AMD"
author = "Orange3-Spark-AMD developers"
extensions = ["myst_parser"]
source_suffix = {".md": "markdown"}
master_doc = "index"
exclude_patterns = ["build"]
html_theme = "alabaster"
