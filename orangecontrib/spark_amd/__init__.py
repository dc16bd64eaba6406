"""Orange3 add-on: MI355X-native replacement for Orange3-Spark's widgets.

Widget logic is headless (see ``widgets/compat.py``); categories "Spark Data (AMD)" and
"Spark ML (AMD)" mirror the reference's "Spark Data" / "Spark ML"
(reference setup.py:17-23).
"""
