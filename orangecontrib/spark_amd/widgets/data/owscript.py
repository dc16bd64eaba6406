"""Python Script widget with the session in scope (reference "PySpark Script",
widgets/data/pyspark_script_console.py:206-466).  A script library is persisted; the
current script runs in a namespace holding ``session``/``spark`` (and the reference's
``sc``/``hc`` aliases), ``in_object`` and ``out_object``; ``out_object`` is READ BACK from
that namespace after execution (the reference sent a stale copy, quirk Q4; the older
working semantics are trash/OLDpyspark_script_console.py:489-492,641-648).

Also as in the reference: an interactive console over the SAME namespace (lines run one
at a time, state persists between lines and with the script, ``out_object`` is read
back; ``code.InteractiveConsole`` semantics of trash/OLDpyspark_script_console.py:125-286)
with the IPython conveniences of the reference's embedded qtconsole
(pyspark_script_console.py:20-29,331): line magics (%time, %timeit, %who, %whos, %reset,
%run, %history, %pwd, %cd, %env, %lsmagic), ``obj?`` / ``obj??`` help, ``!cmd`` and Tab
completion (script_support.ScriptConsole),
"Import a script from a file" / "Save selected script to a file"
(pyspark_script_console.py:286-291,368-392,441-461); the Qt view adds the syntax
highlighter and the auto-indenting editor (script_support.py, ref :39-132)."""
import io
import os
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
        self._console = None

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

    def import_script(self, path: str) -> int:
        """Add the file as a new library entry named after it (ref onAddScriptFromFile)."""
        with open(path, "rb") as f:
            text = f.read().decode("utf-8", errors="ignore")
        self.libraryListSource.append({"name": os.path.basename(path), "script": text,
                                       "filename": os.path.abspath(path)})
        self.currentScriptIndex = len(self.libraryListSource) - 1
        self.scriptText = None
        return self.currentScriptIndex

    def save_script(self, path: str | None = None, index: int | None = None) -> str:
        """Write the selected script (the editor text when it is the current one) to
        ``path`` (default: the file it was imported from / saved to); ``.py`` is added when
        the name has no extension (ref saveScript)."""
        index = self.currentScriptIndex if index is None else index
        entry = self.libraryListSource[index] if 0 <= index < len(self.libraryListSource) else {}
        path = path or entry.get("filename")
        if not path:
            raise ValueError("no file name given for the script")
        if not os.path.splitext(path)[1]:
            path += ".py"
        text = self.current_script() if index == self.currentScriptIndex else entry.get("script", "")
        with open(path, "w", encoding="utf-8") as f:
            f.write(text)
        if entry:
            self.libraryListSource[index] = dict(entry, filename=os.path.abspath(path))
        return path

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

    # -- interactive console -------------------------------------------------------
    def _bind(self):
        ns = self.namespace
        ns.update(session=self.session, spark=self.session, sc=self.sc, hc=self.session,
                  in_object=self.in_object, out_object=self.out_object)
        return ns

    @property
    def console(self):
        from ..script_support import ScriptConsole, banner
        if self._console is None:
            self._console = ScriptConsole(self.namespace, self._console_write, banner(self.session))
        return self._console

    def _console_write(self, data):
        self.console_output += data

    def console_push(self, line: str) -> bool:
        """Run one console line in the widget namespace; True while a block is open."""
        con = self.console
        if not con.more:
            self._bind()
        more = con.push(line)
        self.out_object = self.namespace.get("out_object")
        return more

    def console_paste(self, source: str) -> bool:
        con = self.console
        if not con.more:
            self._bind()
        more = con.paste(source)
        self.out_object = self.namespace.get("out_object")
        return more

    def console_complete(self, text: str) -> list:
        """Completions of the last token of ``text`` (namespace names and attributes, line
        magics) over the widget namespace."""
        if not self.console.more:
            self._bind()
        return self.console.complete(text)

    def console_history(self, step: int) -> str:
        """Previous (step < 0) / next (step > 0) console line."""
        return self.console.history_prev() if step < 0 else self.console.history_next()

    def commit(self):
        ns = self._bind()
        buf = io.StringIO()
        self.error()
        from ..script_support import capture_output
        with capture_output(buf):          # this thread's prints only (the view runs it on a worker)
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
