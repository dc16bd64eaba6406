"""Qt views over the headless widgets, driven through a minimal stand-in for the Orange
widget API (Orange3/Qt are not installed here): signal forwarding, settings sync,
reflective parameter editors, action + output bridging, main-area table."""
import importlib
import pkgutil
import threading
from types import SimpleNamespace

import numpy as np
import pandas as pd
import pytest

from orange3_spark_amd import Session, SessionConf
from orangecontrib.spark_amd.widgets import data as wdata
from orangecontrib.spark_amd.widgets import ml as wml
from orangecontrib.spark_amd.widgets.base import SharedSession
from orangecontrib.spark_amd.widgets.views import export_views, qt_view


def _gui_thread_only(what):
    """The fake Qt objects refuse to be touched off the GUI (main) thread, as Qt requires."""
    if threading.current_thread() is not threading.main_thread():
        raise AssertionError(f"{what} called from worker thread {threading.current_thread().name}")


class _Sig:
    def __init__(self, name, typ, multiple=False):
        self.name, self.type, self.multiple = name, typ, multiple
        self.sent = []

    def __call__(self, fn):                 # Input used as a decorator
        fn._input = self
        return fn

    def send(self, value):
        _gui_thread_only("Output.send")
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
        _gui_thread_only("setHtml")
        self.html = h

    def deleteLater(self):
        pass


class _Signal:
    def __init__(self):
        self.fns = []

    def connect(self, f):
        self.fns.append(f)

    def emit(self, *a):
        for f in self.fns:
            f(*a)


class _Item:
    def __init__(self, t):
        self._t = t

    def text(self):
        return self._t


class _QList(_QW):
    """QListWidget stand-in: items, selection, current row."""

    def __init__(self, *a):
        super().__init__()
        self.sel, self.row = [], -1
        self.currentRowChanged = _Signal()

    def clear(self):
        self.items, self.sel = [], []

    def setSelectionMode(self, m):
        self.mode = m

    def selectedItems(self):
        return [_Item(self.items[i]) for i in self.sel if i < len(self.items)]

    def select(self, *names):                 # test helper: the user's selection
        self.sel = [self.items.index(n) for n in names]

    def setCurrentRow(self, r):
        self.row = r

    def click_row(self, r):                   # test helper: user clicks a row
        self.row = r
        self.currentRowChanged.emit(r)


class _QCombo(_QW):
    def __init__(self, *a):
        super().__init__()
        self.currentTextChanged = _Signal()

    def clear(self):
        self.items = []

    def currentText(self):
        return self.text

    def choose(self, t):                      # test helper
        self.text = t
        self.currentTextChanged.emit(t)


class _QEdit(_QW):
    def __init__(self, text=""):
        super().__init__(text)
        self.textChanged = _Signal()

    def toPlainText(self):
        return self.text

    def setPlainText(self, t):
        self.text = t

    def type(self, t):                        # test helper: the user edits the text
        self.text = t
        self.textChanged.emit()


class _QLine(_QW):
    def __init__(self, text=""):
        super().__init__(text)
        self.textChanged = _Signal()

    def text_(self):
        return self.text


class _QButton(_QW):
    def __init__(self, text=""):
        super().__init__(text)
        self.clicked = _Signal()


class _StateInfo:
    """``OWBaseWidget.info`` in current Orange: the widget's input/output summary object,
    NOT a message method (the messages are ``information`` / ``warning`` / ``error``)."""

    def set_input_summary(self, *a, **k):
        pass

    def set_output_summary(self, *a, **k):
        pass


class _OWWidget:
    def __init__(self, *a, **kw):
        self.controlArea, self.mainArea = _QW(), _QW()
        self.Outputs = type(self).Outputs
        self.shown = {}
        self.info = _StateInfo()
        for cls in type(self).__mro__:           # Setting -> instance default (Orange's SettingProvider)
            for k, v in vars(cls).items():
                if isinstance(v, _Setting) and k not in self.__dict__:
                    setattr(self, k, v.default)

    def error(self, text=None):
        _gui_thread_only("error")
        self.shown["error"] = text

    def information(self, text=None):
        _gui_thread_only("information")
        self.shown["info"] = text

    def warning(self, text=None):
        _gui_thread_only("warning")
        self.shown["warning"] = text

    def onDeleteWidget(self):
        pass


class _Concurrent:
    """Orange's ConcurrentWidgetMixin: ``start(task, *args)`` runs ``task(*args, state)`` on a
    worker thread; progress set on the state is recorded (Orange forwards it to the GUI
    thread's progress bar); ``on_done`` / ``on_exception`` run on the GUI thread."""

    def __init__(self):
        self.progress = []
        self.progress_threads = set()
        self.interrupt = lambda: False        # the Cancel button (Orange: TaskState.interruption)

    def start(self, task, *args):
        state = SimpleNamespace(set_progress_value=self._progress, is_interruption_requested=lambda: self.interrupt())
        box = {}

        def run():
            try:
                box["result"] = task(*args, state)
            except BaseException as e:  # noqa: BLE001 - handed to on_exception like Orange
                box["exc"] = e
        t = threading.Thread(target=run, name="task-worker")
        t.start()
        t.join()
        if "exc" in box:
            self.on_exception(box["exc"])
        else:
            self.on_done(box["result"])

    def _progress(self, p):
        self.progress.append(p)
        self.progress_threads.add(threading.current_thread().name)

    def shutdown(self):
        pass


class _Setting:
    def __init__(self, default):
        self.default = default


def _fake_gui():
    made = []

    def widgetBox(parent, title):
        b = _QW(title)
        made.append(("box", title))
        if hasattr(parent, "layout"):
            parent.layout().addWidget(b)          # Orange adds the box to its parent
        return b

    def checkBox(box, w, attr, label, callback=None):
        made.append(("check", attr, callback))

    def lineEdit(box, w, attr, label=None, callback=None):
        made.append(("line", attr, callback))

    def button(box, w, label, callback=None):
        made.append(("button", label, callback))
    return SimpleNamespace(widgetBox=widgetBox, checkBox=checkBox, lineEdit=lineEdit, button=button, made=made)


class _FakeLineEdit:
    """QLineEdit: text() is a method in Qt."""

    def __init__(self, text=""):
        self._text = text
        self.textChanged = _Signal()
        self.returnPressed = _Signal()

    def setPlaceholderText(self, t):
        self.ph = t

    def enter(self, t):                       # test helper: the user types a line + Return
        self.setText(t)
        self.returnPressed.emit()

    def setToolTip(self, t):
        self.tip = t

    def deleteLater(self):
        pass

    def text(self):
        return self._text

    def setText(self, t):
        self._text = t
        self.textChanged.emit(t)


class _FileDialog:
    """QFileDialog static helpers (Qt5: return (filename, selected_filter))."""
    next_open = next_save = ""

    @staticmethod
    def getOpenFileName(parent, caption, directory, filt):
        return (_FileDialog.next_open, filt)

    @staticmethod
    def getSaveFileName(parent, caption, directory, filt):
        return (_FileDialog.next_save, filt)


@pytest.fixture()
def orange():
    return SimpleNamespace(widget=SimpleNamespace(OWWidget=_OWWidget, Input=_Sig, Output=_Sig),
                           settings=SimpleNamespace(Setting=_Setting), gui=_fake_gui(),
                           qt=SimpleNamespace(QTextBrowser=_QEdit, QLabel=_QW, QComboBox=_QCombo, QLineEdit=_FakeLineEdit,
                                              QListWidget=_QList, QPushButton=_QButton, QPlainTextEdit=_QEdit,
                                              QFileDialog=_FileDialog,
                                              QAbstractItemView=SimpleNamespace(ExtendedSelection=3)),
                           concurrent=None)


@pytest.fixture()
def orange_mt(orange):
    """The same stand-ins with Orange's ConcurrentWidgetMixin: actions on a worker thread."""
    orange.concurrent = _Concurrent
    return orange


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



def _click(view, label):
    for box in _all_widgets(view):
        if isinstance(box, _QButton) and box.text == label:
            box.clicked.emit()
            return
    raise KeyError(label)


def _all_widgets(view):
    out = []
    for root in (view.controlArea, view.mainArea):
        stack = [root]
        while stack:
            w = stack.pop()
            out.append(w)
            stack.extend(w.layout().items if hasattr(w, "layout") else [])
    return out


def test_dataset_builder_view_assigns_roles_through_its_controls(orange, session, monkeypatch):
    """Role assignment from the canvas: select columns in the list views, press the move
    buttons, reorder, filter -- then Commit assembles exactly those features."""
    import orangecontrib.spark_amd.widgets.custom_views as CV
    from orangecontrib.spark_amd.widgets.ml.owdatasetbuilder import OWDatasetBuilder
    made = []
    orig = CV.build_dataset_builder

    def spy(view, o):
        r = orig(view, o)
        made.append(view)
        return r
    monkeypatch.setitem(CV.BUILDERS, "OWDatasetBuilder", spy)
    V = qt_view(OWDatasetBuilder, orange)
    w = V()
    lists = w.builder_lists
    df = session.createDataFrame(pd.DataFrame({"x1": [1.0, 2.0, 3.0], "x2": [4.0, 5.0, 6.0], "x3": [7.0, 8.0, 9.0],
                                               "y": [0, 1, 0], "note": ["a", "b", "c"]}))
    w.set_dataframe(df)
    assert lists["available"].items == ["x1", "x2", "x3", "y", "note"]
    lists["filter"].setText("x")                         # filter narrows the available list
    assert lists["available"].items == ["x1", "x2", "x3"]
    lists["available"].select("x1", "x3")
    _click(w, "Features >")
    lists["filter"].setText("")
    lists["available"].select("y")
    _click(w, "Label >")
    lists["available"].select("note")
    _click(w, "Meta >")
    lists["available"].select("x2")
    _click(w, "Features >")
    lists["features"].select("x2")
    _click(w, "Up")                                      # features now x1, x2, x3
    assert lists["features"].items == ["x1", "x2", "x3"] and lists["label"].items == ["y"]
    assert lists["metas"].items == ["note"] and lists["available"].items == []
    lists["features"].select("x3")
    _click(w, "< Available")
    assert lists["available"].items == ["x3"]
    w.run_action()
    out = V.Outputs.dataframe.sent[-1]
    rows = out.select("features", "label").collect()
    assert [list(r.features.toArray()) for r in rows] == [[1.0, 4.0], [2.0, 5.0], [3.0, 6.0]]
    assert [r.label for r in rows] == [0.0, 1.0, 0.0]
    assert "note" in out.columns
    # the role hints were persisted into the widget setting (workflow save)
    assert w.domain_role_hints


def test_catalog_table_view_combo_boxes(orange, session, tmp_path):
    from orangecontrib.spark_amd.widgets.data.owtable import OWCatalogTable
    session.sql("CREATE DATABASE IF NOT EXISTS sales")
    session.createDataFrame(pd.DataFrame({"a": [1, 2]})).write.mode("overwrite").saveAsTable("sales.q1")
    session.createDataFrame(pd.DataFrame({"a": [3, 4, 5]})).write.mode("overwrite").saveAsTable("sales.q2")
    V = qt_view(OWCatalogTable, orange)
    w = V()
    c = w.table_controls
    w._refresh_editors()
    assert "default" in c["databases"].items and "sales" in c["databases"].items
    c["databases"].choose("sales")                       # database combo -> table combo refilled
    assert set(c["tables"].items) == {"q1", "q2"} and w.database == "sales"
    c["tables"].choose("q2")
    assert w.table == "q2"
    w.run_action()                                       # Submit
    assert V.Outputs.dataframe.sent[-1].count() == 3
    assert not any(m[:2] == ("line", "table") for m in orange.gui.made)   # combo, not a line edit


def test_script_view_library_editor_and_console(orange, session):
    from orangecontrib.spark_amd.widgets.data.owscript import OWScript
    V = qt_view(OWScript, orange)
    w = V()
    sc = w.script_controls
    w._refresh_editors()
    assert sc["library"].items == ["Hello session"] and "out_object = in_object" in sc["editor"].text
    sc["editor"].type("out_object = 6 * 7\nprint('answer', out_object)")
    _click(w, "+")                                        # save as a new library entry
    assert sc["library"].items == ["Hello session", "Script 2"] and w.core.currentScriptIndex == 1
    w.run_action()
    assert V.Outputs.out_object.sent[-1] == 42
    assert "answer 42" in sc["console"].text
    sc["library"].click_row(0)                            # back to the first script
    assert sc["editor"].text.startswith("out_object = in_object")
    sc["editor"].type("out_object = 'changed'")
    _click(w, "Update")
    assert w.core.libraryListSource[0]["script"] == "out_object = 'changed'"
    _click(w, "-")
    assert sc["library"].items == ["Script 2"]


def test_script_view_console_import_and_save(orange, session, tmp_path):
    from orangecontrib.spark_amd.widgets.data.owscript import OWScript
    V = qt_view(OWScript, orange)
    w = V()
    sc = w.script_controls
    w._refresh_editors()
    sc["console_input"].enter("x = 20")
    sc["console_input"].enter("out_object = x + 1")
    assert w.core.out_object == 21 and ">>> out_object = x + 1" in sc["console"].text
    src = tmp_path / "job.py"
    src.write_text("out_object = x * 2\n")
    _FileDialog.next_open = str(src)
    _click(w, "Import a script from a file")
    assert sc["library"].items[-1] == "job.py" and sc["editor"].text == "out_object = x * 2\n"
    w.run_action()                                        # the script sees the console's x
    assert V.Outputs.out_object.sent[-1] == 40
    sc["editor"].type("out_object = 'saved'\n")
    _FileDialog.next_save = str(tmp_path / "copy")
    _click(w, "Save selected script to a file")
    assert (tmp_path / "copy.py").read_text() == "out_object = 'saved'\n"


def test_tutorial_names_are_the_classes_orange_registers(orange):
    """Every node of the shipped tutorial names a Qt view class that export_views creates
    in that module (what Orange's discovery registers), and the headless runner resolves
    it to the widget's core."""
    import importlib
    import os
    import xml.etree.ElementTree as ET
    from orangecontrib.spark_amd.workflow import resolve
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    ows = os.path.join(root, "orangecontrib", "spark_amd", "tutorials", "spark_ml.ows")
    names = [n.get("qualified_name") for n in ET.parse(ows).getroot().iter("node")]
    assert len(names) == 8
    for qn in names:
        mod, _, cls = qn.rpartition(".")
        assert cls.endswith("View")
        g = dict(vars(importlib.import_module(mod)))
        views = {v.__qualname__: v for v in export_views(g, orange)}
        assert cls in views, qn
        assert resolve(qn) is views[cls].core_class


def test_concurrent_fit_reports_progress_and_touches_qt_only_on_gui_thread(orange_mt, session):
    """Q14 intent (reference spark_ml_estimator.py:19-25 froze the GUI): the Apply action
    runs the fit on a worker thread, the 20-iteration LR fit's progress rises
    monotonically to 100 on the task state, and every Qt mutation (outputs, messages,
    the main-area table) happens on the GUI thread -- the fakes raise otherwise."""
    from orangecontrib.spark_amd.widgets.ml.owclassification import OWClassification
    V = qt_view(OWClassification, orange_mt)
    w = V()
    df = session.createDataFrame(pd.DataFrame({"features": [[0.0, 1.0], [1.0, 0.3], [0.2, 0.9], [0.8, 0.1]] * 50,
                                               "label": [1.0, 0.0, 1.0, 0.0] * 50}))
    w._param_changed("method", "LogisticRegression")
    w.set_dataframe(df)
    w._param_changed("maxIter", "20")
    w._param_changed("tol", "0.0")
    w.run_action()
    model = V.Outputs.model.sent[-1]
    assert type(model).__name__ == "LogisticRegressionModel"
    p = w.progress
    assert len(p) >= 10 and p[-1] == 100.0 and all(b >= a for a, b in zip(p, p[1:])), p
    assert w.progress_threads == {"task-worker"}
    w.core.info("done on the worker")                    # GUI-thread call: shown at once
    assert w.shown["info"] == "done on the worker"


@pytest.mark.timeout(300)
def test_pool_fit_from_the_view_reports_progress_and_cancels(orange_mt):
    """The 8-GPU canvas deployment in miniature: the Context is a 2-executor pool, the
    Classification view's Apply runs the fit on a worker thread, rank 0's per-iteration
    progress reaches the task state, and Cancel stops the fit on every executor at the
    same iteration -- the widget shows FitCancelled, the pool survives for the next Apply."""
    from orangecontrib.spark_amd.widgets.ml.owclassification import OWClassification
    pool = Session(SessionConf().set("spark.executor.instances", "2").set("o3s.device", "cpu"))
    prev = SharedSession._session
    SharedSession._session = pool
    try:
        V = qt_view(OWClassification, orange_mt)
        w = V()
        rng = np.random.default_rng(0)
        X = rng.normal(size=(4000, 2))
        df = pool.createDataFrame(pd.DataFrame({"features": list(X), "label": (X[:, 0] > X[:, 1]).astype(float)}))
        w._param_changed("method", "LogisticRegression")
        w.set_dataframe(df)
        w._param_changed("solver", "sgd")
        w._param_changed("maxIter", "20")
        w._param_changed("tol", "0.0")
        w.run_action()
        assert type(V.Outputs.model.sent[-1]).__name__ == "LogisticRegressionModel"
        p = list(w.progress)
        assert len(p) >= 15 and p[-1] == 100.0 and all(b >= a for a, b in zip(p, p[1:])), p
        pids = list(pool.pool.pids)
        w.progress.clear()
        sent = len(V.Outputs.model.sent)
        w._param_changed("maxIter", "400")
        w.interrupt = lambda: bool(w.progress) and w.progress[-1] >= 50.0
        w.run_action()
        assert "FitCancelled" in (w.shown.get("error") or "")
        assert len(V.Outputs.model.sent) == sent and w.progress[-1] < 52.0
        assert pool.pool.alive and pool.pool.pids == pids
        w.interrupt = lambda: False
        w._param_changed("maxIter", "5")
        w.run_action()
        assert len(V.Outputs.model.sent) == sent + 1
    finally:
        SharedSession._session = prev
        pool.stop()


def test_worker_messages_are_queued_to_the_gui_thread(orange_mt, session):
    """A message raised by the action on the worker (the Context widget's device list, an
    estimator's warning) is delivered by the GUI thread when the task ends, through
    ``information`` (``info`` is the StateInfo summary in current Orange)."""
    from orangecontrib.spark_amd.widgets.data.owcontext import OWSessionContext
    V = qt_view(OWSessionContext, orange_mt)
    w = V()
    w.core.set_param("o3s.device", "cpu")
    w.run_action()
    try:
        assert "device" in (w.shown.get("info") or "") and isinstance(w.info, _StateInfo)
    finally:
        w.core.onDeleteWidget()
        SharedSession._session = session


def test_script_on_worker_captures_only_its_own_prints(orange_mt, session, capsys):
    """The Script widget's commit runs on the worker: its prints go to the console, a
    print from another thread while it runs does NOT (no process-global redirect)."""
    from orangecontrib.spark_amd.widgets.data.owscript import OWScript
    V = qt_view(OWScript, orange_mt)
    w = V()
    sc = w.script_controls
    w._refresh_editors()
    other = threading.Event()

    def bystander():
        print("bystander line")
        other.set()
    import orangecontrib.spark_amd.widgets.data.owscript as mod
    mod._test_hook = bystander
    sc["editor"].type("import threading, orangecontrib.spark_amd.widgets.data.owscript as m\n"
                      "t = threading.Thread(target=m._test_hook); t.start(); t.join()\n"
                      "print('from the script')\nout_object = 5")
    w.run_action()
    assert V.Outputs.out_object.sent[-1] == 5 and other.is_set()
    assert "from the script" in sc["console"].text and "bystander line" not in sc["console"].text
    assert "bystander line" in capsys.readouterr().out


def test_view_settings_do_not_share_the_headless_default(orange):
    """A Qt view's setting default is a copy of the headless widget's: editing a view
    instance's saved parameters in place must not change later headless widgets (it made
    the Context widget's editor show a stale saved seed in another test)."""
    from orangecontrib.spark_amd.widgets.data import owcontext
    from orangecontrib.spark_amd.widgets.views import qt_view
    core = owcontext.OWSessionContext.saved_gui_params
    V = qt_view(owcontext.OWSessionContext, orange)
    assert V.saved_gui_params.default == core.default
    assert V.saved_gui_params.default is not core.default
    V.saved_gui_params.default["o3s.seed"] = "42"
    assert "o3s.seed" not in core.default
