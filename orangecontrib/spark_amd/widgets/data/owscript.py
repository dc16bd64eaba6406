"""Python Script widget with the session in scope (reference "PySpark Script",
widgets/data/pyspark_script_console.py:206-466).  A script library is persisted; the
current script runs in a namespace holding ``session``/``spark`` (and the reference's
``sc``/``hc`` aliases), ``in_object`` and ``out_object``; ``out_object`` is READ BACK from
that namespace after execution (the reference sent a stale copy, quirk Q4; the older
working semantics are trash/OLDpyspark_script_console.py:489-492,641-648)."""
import contextlib
import io
import traceback

from ..base import SharedSession
from ..compat import Setting, Widget


class OWScript(SharedSession, Widget):
    priority = 3
    name = "Python Script"
    description = "Run Python against the shared session; in_object -> out_object"
    icon = "../icons/python.svg"
    inputs = [("in_object", object, "set_in_object")]
    outputs = [("out_object", object)]
    libraryListSource = Setting([{"name": "Hello session", "script": "out_object = in_object\n"
                                                                    "print(session)"}])
    currentScriptIndex = Setting(0)
    scriptText = Setting(None)
    auto_commit = Setting(True)

    def __init__(self, **kw):
        super().__init__(**kw)
        self.in_object = None
        self.out_object = None
        self.console_output = ""
        self.namespace = {}

    # -- library ---------------------------------------------------------------
    def add_script(self, name, script):
        self.libraryListSource.append({"name": name, "script": script})
        self.currentScriptIndex = len(self.libraryListSource) - 1

    def remove_script(self, index):
        del self.libraryListSource[index]
        self.currentScriptIndex = max(0, min(self.currentScriptIndex, len(self.libraryListSource) - 1))

    def select_script(self, index):
        """Show library entry ``index`` in the editor (discarding unsaved edits)."""
        if 0 <= index < len(self.libraryListSource):
            self.currentScriptIndex = index
            self.scriptText = None

    def update_script(self, index, script):
        """Store the editor text into library entry ``index``."""
        if 0 <= index < len(self.libraryListSource):
            self.libraryListSource[index] = dict(self.libraryListSource[index], script=script)
            self.scriptText = None

    def current_script(self) -> str:
        if self.scriptText is not None:
            return self.scriptText
        return self.libraryListSource[self.currentScriptIndex]["script"] if self.libraryListSource else ""

    # -- signals ---------------------------------------------------------------
    def set_in_object(self, obj):
        self.in_object = obj

    def handleNewSignals(self):
        if self.auto_commit:
            self.commit()

    def commit(self):
        ns = self.namespace
        ns.update(session=self.session, spark=self.session, sc=self.sc, hc=self.session,
                  in_object=self.in_object, out_object=self.out_object)
        buf = io.StringIO()
        self.error()
        with contextlib.redirect_stdout(buf), contextlib.redirect_stderr(buf):
            try:
                exec(compile(self.current_script(), "<script>", "exec"), ns)
            except Exception:  # noqa: BLE001
                traceback.print_exc()
                self.error("script raised an exception (see console output)")
        self.console_output += buf.getvalue()
        self.out_object = ns.get("out_object")
        self.send("out_object", self.out_object)
        return self.out_object


from ..views import export_views  # noqa: E402

export_views(globals())
