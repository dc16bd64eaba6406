"""Qt views over the headless widgets, driven through a minimal stand-in for the Orange
widget API (Orange3/Qt are not installed here): signal forwarding, settings sync,
reflective parameter editors, action + output bridging, main-area table."""
import importlib
import pkgutil
from types import SimpleNamespace

import pandas as pd
import pytest

from orange3_spark_amd import Session, SessionConf
from orangecontrib.spark_amd.widgets import data as wdata
from orangecontrib.spark_amd.widgets import ml as wml
from orangecontrib.spark_amd.widgets.base import SharedSession
from orangecontrib.spark_amd.widgets.views import export_views, qt_view


class _Sig:
    def __init__(self, name, typ, multiple=False):
        self.name, self.type, self.multiple = name, typ, multiple
        self.sent = []

    def __call__(self, fn):                 # Input used as a decorator
        fn._input = self
        return fn

    def send(self, value):
        self.sent.append(value)


class _Layout:
    def __init__(self):
        self.items = []

    def addWidget(self, w):
        self.items.append(w)

    def count(self):
        return len(self.items)

    def takeAt(self, i):
        w = self.items.pop(i)
        return SimpleNamespace(widget=lambda: w)


class _QW:
    def __init__(self, text=""):
        self.text, self.items, self.tip, self.html = text, [], None, None
        self._layout = _Layout()
        self.currentTextChanged = self.textChanged = SimpleNamespace(connect=lambda f: setattr(self, "cb", f))

    def layout(self):
        return self._layout

    def addItems(self, xs):
        self.items += xs

    def setCurrentText(self, t):
        self.text = t

    def setToolTip(self, t):
        self.tip = t

    def setPlaceholderText(self, t):
        self.ph = t

    def setHtml(self, h):
        self.html = h

    def deleteLater(self):
        pass


class _OWWidget:
    def __init__(self, *a, **kw):
        self.controlArea, self.mainArea = _QW(), _QW()
        self.Outputs = type(self).Outputs
        self.shown = {}
        for cls in type(self).__mro__:           # Setting -> instance default (Orange's SettingProvider)
            for k, v in vars(cls).items():
                if isinstance(v, _Setting) and k not in self.__dict__:
                    setattr(self, k, v.default)

    def error(self, text=None):
        self.shown["error"] = text

    def info(self, text=None):
        self.shown["info"] = text

    def warning(self, text=None):
        self.shown["warning"] = text

    def onDeleteWidget(self):
        pass


class _Setting:
    def __init__(self, default):
        self.default = default


def _fake_gui():
    made = []

    def widgetBox(parent, title):
        b = _QW(title)
        made.append(("box", title))
        return b

    def checkBox(box, w, attr, label, callback=None):
        made.append(("check", attr, callback))

    def lineEdit(box, w, attr, label=None, callback=None):
        made.append(("line", attr, callback))

    def button(box, w, label, callback=None):
        made.append(("button", label, callback))
    return SimpleNamespace(widgetBox=widgetBox, checkBox=checkBox, lineEdit=lineEdit, button=button, made=made)


@pytest.fixture()
def orange():
    return SimpleNamespace(widget=SimpleNamespace(OWWidget=_OWWidget, Input=_Sig, Output=_Sig),
                           settings=SimpleNamespace(Setting=_Setting), gui=_fake_gui(),
                           qt=SimpleNamespace(QTextBrowser=_QW, QLabel=_QW, QComboBox=_QW, QLineEdit=_QW),
                           concurrent=None)


@pytest.fixture(scope="module")
def session():
    s = Session(SessionConf().set("o3s.device", "cpu"))
    SharedSession._session = s
    yield s
    SharedSession._session = None


def test_every_widget_module_gets_a_view(orange):
    n = 0
    for pkg in (wdata, wml):
        for info in pkgutil.iter_modules(pkg.__path__):
            mod = importlib.import_module(f"{pkg.__name__}.{info.name}")
            g = dict(vars(mod))
            views = export_views(g, orange)
            assert views, info.name
            for v in views:
                assert v.__module__ == mod.__name__ and v.name == v.core_class.name
            n += len(views)
    assert n >= 25


def test_sample_view_forwards_signals_and_settings(orange, session):
    from orangecontrib.spark_amd.widgets.data.owsample import OWSample
    V = qt_view(OWSample, orange)
    w = V()
    assert any(m[:2] == ("line", "fraction") for m in orange.gui.made)
    df = session.createDataFrame(pd.DataFrame({"a": range(1000)}))
    w.set_dataframe(df)
    w.fraction = "0.25"
    w.run_action()                                    # Apply: settings synced, output bridged
    out = V.Outputs.dataframe.sent[-1]
    assert 150 < out.count() < 350
    labels = [m[1] for m in orange.gui.made if m[0] == "button"]
    assert "Apply" in labels


def test_reflective_estimator_view_builds_param_editors(orange, session):
    from orangecontrib.spark_amd.widgets.ml.owclassification import OWClassification
    V = qt_view(OWClassification, orange)
    w = V()
    lay = w._param_box.layout()
    assert any(getattr(x, "items", None) and "LogisticRegression" in x.items for x in lay.items)
    w._param_changed("method", "LinearSVC")
    assert w.core.method.__name__ == "LinearSVC" and "regParam" in w.core.gui_parameters
    df = session.createDataFrame(pd.DataFrame({"features": [[0.0, 1.0], [1.0, 0.0]] * 20, "label": [1.0, 0.0] * 20}))
    w.set_dataframe(df)
    w._param_changed("maxIter", "5")
    w.run_action()
    model = V.Outputs.model.sent[-1]
    assert type(model).__name__ == "LinearSVCModel"
    assert w.saved_gui_params["method"] == "LinearSVC"       # synced back into the Qt setting


def test_evaluation_view_shows_metric_table_and_errors(orange, session):
    from orangecontrib.spark_amd.widgets.ml.owevaluation import OWEvaluation
    V = qt_view(OWEvaluation, orange)
    w = V()
    assert V.want_main_area and w.result_view is not None
    df = session.createDataFrame(pd.DataFrame({"prediction": [1.0, 2.0, 3.0], "label": [1.0, 2.0, 4.0]}))
    w._param_changed("method", "RegressionEvaluator")
    w.set_dataframe(df)
    w.run_action()
    assert "rmse" in w.result_view.html
    w.core.error("boom")
    assert w.shown["error"] == "boom"
