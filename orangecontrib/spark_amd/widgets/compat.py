"""Headless widget runtime, API-compatible with the subset of Orange3's widget framework
the reference uses (``OWWidget`` class attributes, old-style ``inputs``/``outputs``
tuples, ``Setting``, ``self.send(channel, obj)``, ``info/warning/error``).

Orange3 and Qt are not installed here, so every widget's logic is written
against this module and is fully testable headlessly; :mod:`.workflow` wires widgets into
a signal graph (the canvas) and replays ``.ows`` files.  When Orange *is* importable,
``HAVE_ORANGE`` is True and :mod:`.views` wraps every headless widget in a generated
Qt ``OWWidget`` subclass (``<Class>View``) that Orange's widget discovery finds.
"""
from __future__ import annotations

import copy
import logging
from collections import OrderedDict

try:  # pragma: no cover - exercised only with Orange installed
    import Orange.widgets.widget  # noqa: F401
    HAVE_ORANGE = True
except Exception:  # noqa: BLE001
    HAVE_ORANGE = False

log = logging.getLogger("orangecontrib.spark_amd")

# signal flags (Orange's widget.Default / Dynamic / Multiple / Explicit)
Default, Dynamic, Multiple, Explicit, Single = 1, 2, 4, 8, 16


class Setting:
    """Persisted widget attribute (copied per instance, stored in workflow properties)."""

    def __init__(self, default, **kw):
        self.default = default
        self.kw = kw

    def __repr__(self):
        return f"Setting({self.default!r})"


class _Message:
    def __init__(self):
        self.text = None

    def __call__(self, text=None, *a, **k):
        self.text = text

    def clear(self):
        self.text = None


class Widget:
    """Headless OWWidget: name/description/icon/priority metadata, signals, settings."""

    name = "Widget"
    description = ""
    icon = ""
    priority = 100
    category = None
    inputs: list = []
    outputs: list = []
    want_main_area = False
    resizing_enabled = True

    def __init__(self, **settings):
        self._settings = OrderedDict()
        for k in dir(type(self)):
            v = getattr(type(self), k, None)
            if isinstance(v, Setting):
                val = copy.deepcopy(v.default)
                if k in settings:
                    val = settings.pop(k)
                object.__setattr__(self, k, val)
                self._settings[k] = True
        self.sent = OrderedDict()          # channel -> last value sent
        self.signal_manager = None
        self.messages = {"info": None, "warning": None, "error": None}
        self.visible = True
        for k, v in settings.items():
            setattr(self, k, v)

    # -- signals ---------------------------------------------------------------
    def send(self, channel: str, value):
        names = [o[0] for o in self.outputs]
        if channel not in names:
            raise ValueError(f"{type(self).__name__} has no output channel {channel!r}")
        self.sent[channel] = value
        if self.signal_manager is not None:
            self.signal_manager.send(self, channel, value)

    def handleNewSignals(self):
        pass

    # -- messages ---------------------------------------------------------------
    def info(self, text=None):
        self.messages["info"] = text

    def warning(self, text=None):
        self.messages["warning"] = text

    def error(self, text=None):
        self.messages["error"] = text
        if text:
            log.error("%s: %s", self.name, text)

    # -- settings ---------------------------------------------------------------
    def settings_dict(self) -> dict:
        return {k: copy.deepcopy(getattr(self, k)) for k in self._settings}

    def apply_settings(self, d: dict):
        for k, v in (d or {}).items():
            if k in self._settings:
                setattr(self, k, v)

    def hide(self):
        self.visible = False

    def show(self):
        self.visible = True

    def onDeleteWidget(self):
        pass

    # -- helpers for subclasses -----------------------------------------------------
    @classmethod
    def input_handler(cls, channel: str) -> str:
        for inp in cls.inputs:
            if inp[0] == channel:
                return inp[2]
        raise KeyError(channel)


class SignalManager:
    """Minimal canvas: links (src, out_channel) -> (dst, in_channel); synchronous delivery."""

    def __init__(self):
        self.widgets = []
        self.links = []

    def add(self, w: Widget) -> Widget:
        w.signal_manager = self
        self.widgets.append(w)
        return w

    def link(self, src: Widget, out_ch: str, dst: Widget, in_ch: str):
        self.links.append((src, out_ch, dst, in_ch))
        if out_ch in src.sent:           # late link: deliver the current value
            self._deliver(dst, in_ch, src.sent[out_ch])

    def send(self, src, channel, value):
        for s, oc, d, ic in self.links:
            if s is src and oc == channel:
                self._deliver(d, ic, value)

    @staticmethod
    def _deliver(dst, in_ch, value):
        handler = getattr(dst, dst.input_handler(in_ch))
        handler(value)
        dst.handleNewSignals()
