"""Headless parameter editor with the reference's exact string->value coercion.

Reference: orangecontrib/spark/utils/gui_utils.py (GuiParam, :5-103).  The editor keeps
the raw string (``get_value``) and converts it with ``get_usable_value`` using the same
rules (:78-94): 'None'/'' -> None; 'True'/'False' -> bool; integer literal -> int; other
numeric -> float; otherwise the string.  Beyond the reference (quirk Q11): a value of the
form ``[a, b, ...]`` is parsed into a list with each element coerced by the same rules,
so array-typed Params (inputCols, thresholds, splits) become settable.
"""
from __future__ import annotations


def coerce(val):
    if val is None:
        return None
    val = str(val).strip()
    if val == "None" or val == "":
        return None
    if val in ("True", "False"):
        return val == "True"
    if val.startswith("[") and val.endswith("]"):
        inner = val[1:-1].strip()
        if not inner:
            return []
        return [coerce(p.strip().strip("'\"")) for p in inner.split(",")]
    try:
        try:
            if float(val) == int(val):
                if "." in val:
                    return float(val)
                return int(val)
        except ValueError:
            return float(val)
    except ValueError:
        return val
    return float(val)


class GuiParam:
    """One labelled parameter editor (combo box when ``list_values`` is given, or
    automatically True/False when the default is the string 'True'/'False')."""

    def __init__(self, parent_widget=None, label=None, default_value=None, place_holder_text=None, list_values=None,
                 callback_func=None, doc_text=None, **kwargs):
        self.default_value = default_value
        if default_value in ("True", "False"):
            list_values = ["True", "False"]
        self.list_values = list(list_values) if list_values else None
        self.gui_type = "multiple" if self.list_values else "single"
        self.label = (label + ":") if label else None
        self.place_holder_text = place_holder_text
        self.doc_text = doc_text
        self.callback_func = callback_func
        self.parent_widget = parent_widget
        if self.gui_type == "multiple":
            if default_value is not None and str(default_value) in self.list_values:
                self._value = str(default_value)
            else:
                self._value = self.list_values[0]
        else:
            self._value = "" if default_value is None else str(default_value)

    def get_value(self) -> str:
        return self._value

    def set_value(self, value) -> None:
        v = "" if value is None else str(value)
        if self.gui_type == "multiple" and v not in self.list_values:
            raise ValueError(f"{v!r} is not one of {self.list_values}")
        self._value = v
        if self.callback_func and self.gui_type == "multiple":
            self.callback_func(v)

    def update(self, values) -> None:
        if self.gui_type == "multiple":
            self.list_values = list(values)
            if self._value not in self.list_values and self.list_values:
                self._value = self.list_values[0]
        else:
            self._value = str(values)

    def get_usable_value(self):
        return coerce(self.get_value())

    def __repr__(self):
        return f"GuiParam({self.label!r}, {self._value!r})"
