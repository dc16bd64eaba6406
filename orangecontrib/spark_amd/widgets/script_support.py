"""Python-script tooling of the Script widget, Qt-free so it is testable headless.

Reference: orangecontrib/spark/widgets/data/pyspark_script_console.py --
``PythonSyntaxHighlighter`` (:39-97), ``PythonScriptEditor`` auto-indent (:100-132) and the
interactive console.  The console follows the reference's older, working
``PySparkConsole`` (trash/OLDpyspark_script_console.py:125-286): a
``code.InteractiveConsole`` over the widget namespace, so lines typed there see and set
``out_object``, with history and multi-line paste.  The Qt view (custom_views.py) wraps
these in a ``QSyntaxHighlighter`` subclass, a ``QPlainTextEdit`` with the indent keys
and an input line under the console pane.
"""
from __future__ import annotations

import code
import contextlib
import keyword
import re
import sys
import threading

INDENT = 4

# -------------------------------------------------------------------------- highlighter
# span formats (the Qt view maps them to QTextCharFormat: colour, weight)
FORMATS = {"keyword": ("blue", True), "def": ("black", True), "string": ("darkGreen", False),
           "comment": ("lightGray", False), "decorator": ("darkGray", False), "number": ("darkMagenta", False)}

_RULES = [(re.compile(r"\b(?:%s)\b" % "|".join(keyword.kwlist)), "keyword", 0),
          (re.compile(r"\bdef\s+([A-Za-z_][A-Za-z0-9_]*)\s*\("), "def", 1),
          (re.compile(r"\bclass\s+([A-Za-z_][A-Za-z0-9_]*)\s*[(:]"), "def", 1),
          (re.compile(r"\b\d+(?:\.\d*)?(?:[eE][-+]?\d+)?\b"), "number", 0),
          (re.compile(r"@[A-Za-z_][A-Za-z0-9_.]*"), "decorator", 0)]
_STRING = re.compile(r"'(?:[^'\\]|\\.)*'|\"(?:[^\"\\]|\\.)*\"")
_TRIPLE = re.compile(r"'''|\"\"\"")


def highlight_spans(text: str, prev_state: int = 0):
    """Spans ``[(start, length, format)]`` of one line and the block state to carry into
    the next line (1 = inside a triple-quoted string opened by ``'''`` , 2 = by
    ``\"\"\"``).  Later spans override earlier ones (QSyntaxHighlighter.setFormat order):
    rules, then strings, then comments, then triple-quoted strings."""
    spans = []
    for rx, fmt, grp in _RULES:
        for m in rx.finditer(text):
            spans.append((m.start(grp), m.end(grp) - m.start(grp), fmt))
    comment_at = None
    for m in _STRING.finditer(text):
        spans.append((m.start(), m.end() - m.start(), "string"))
    # a '#' outside any string starts a comment
    masked = _STRING.sub(lambda m: " " * (m.end() - m.start()), text)
    i = masked.find("#")
    if i >= 0:
        comment_at = i
        spans.append((i, len(text) - i, "comment"))
    state, pos = prev_state, 0
    if state:                                   # continue an open triple-quoted string
        close = "'''" if state == 1 else '"""'
        j = text.find(close)
        if j < 0:
            return [(0, len(text), "string")], state
        spans.append((0, j + 3, "string"))
        pos, state = j + 3, 0
    while True:
        m = _TRIPLE.search(text, pos)
        if m is None or (comment_at is not None and m.start() > comment_at):
            break
        q = m.group(0)
        j = text.find(q, m.end())
        if j < 0:
            spans.append((m.start(), len(text) - m.start(), "string"))
            return spans, 1 if q == "'''" else 2
        spans.append((m.start(), j + 3 - m.start(), "string"))
        pos = j + 3
    return spans, 0


# ------------------------------------------------------------------------------- editor
def indent_after(line: str) -> int:
    """Indent (spaces) of the line opened by Return after ``line`` (reference
    PythonScriptEditor.keyPressEvent: keep the indent, +4 after ':', -4 after ``pass`` /
    ``return``)."""
    indent = len(line) - len(line.lstrip(" "))
    st = line.strip()
    if st == "pass" or st.startswith("return ") or st == "return" or st in ("break", "continue") \
            or st.startswith("raise "):
        return max(0, indent - INDENT)
    if st.endswith(":") and not st.startswith("#"):
        return indent + INDENT
    return indent


def backspace_width(line_before_cursor: str) -> int:
    """Characters one Backspace deletes: a whole indent step inside leading blanks."""
    if line_before_cursor and not line_before_cursor.strip():
        return min(INDENT, len(line_before_cursor)) or 1
    return 1


# ------------------------------------------------------------------------------ console
class ScriptConsole(code.InteractiveConsole):
    """Interactive interpreter over a shared namespace.  ``push`` runs one line (returns
    True while a block is incomplete); everything printed goes to ``write``; a transcript
    with ``>>> `` / ``... `` prompts is kept as the console text."""

    def __init__(self, namespace: dict, write, banner: str | None = None):
        super().__init__(namespace, filename="<console>")
        self._write = write
        self.history: list[str] = []
        self._hpos = 0
        self.more = False
        if banner:
            self.write(banner if banner.endswith("\n") else banner + "\n")

    @property
    def prompt(self) -> str:
        return "... " if self.more else ">>> "

    def write(self, data):
        self._write(data)

    def push(self, line: str) -> bool:
        self.write(self.prompt + line + "\n")
        if line.strip() and (not self.history or self.history[-1] != line):
            self.history.append(line)
        self._hpos = len(self.history)
        out = _Writer(self.write)
        with capture_output(out):
            try:
                if not self.more and self._special(line):
                    return self.more
                self.more = bool(super().push(line))
            except SystemExit:
                self.resetbuffer()
                self.more = False
        return self.more

    # ---- IPython conveniences (the reference embeds an IPython kernel, qtconsole:
    # pyspark_script_console.py:20-29,331; none is importable here, so the usual line
    # magics, ``obj?`` help, ``!cmd`` and completion are implemented over this namespace) --
    MAGICS = ("cd", "env", "history", "lsmagic", "pwd", "reset", "run", "time", "timeit", "who", "whos")
    _HELP = re.compile(r"^\s*([A-Za-z_][\w.]*)\s*(\?\??)\s*$")

    def _special(self, line: str) -> bool:
        """Run ``line`` if it is a magic, a help request or a shell escape; False if it is
        plain Python."""
        s = line.strip()
        if s.startswith("%"):
            name, _, arg = s[1:].partition(" ")
            fn = getattr(self, "_magic_" + name, None)
            if fn is None:
                print(f"UsageError: Line magic function `%{name}` not found.")
            else:
                try:
                    fn(arg.strip())
                except Exception:  # noqa: BLE001
                    self.showtraceback()
            return True
        if s.startswith("!"):
            import subprocess
            r = subprocess.run(s[1:], shell=True, capture_output=True, text=True)
            print((r.stdout + r.stderr).rstrip("\n"))
            return True
        m = self._HELP.match(line)
        if m:
            self._help(m.group(1), m.group(2) == "??")
            return True
        return False

    def _eval(self, expr: str):
        return eval(expr, self.locals)

    def _help(self, expr: str, source: bool) -> None:
        import inspect
        try:
            obj = self._eval(expr)
        except Exception as e:  # noqa: BLE001
            print(f"Object `{expr}` not found ({type(e).__name__}).")
            return
        print(f"Type:      {type(obj).__name__}")
        try:
            print(f"Signature: {expr}{inspect.signature(obj)}")
        except (TypeError, ValueError):
            pass
        if source:
            try:
                print(inspect.getsource(obj))
                return
            except (TypeError, OSError):
                pass
        doc = inspect.getdoc(obj)
        print("Docstring:", doc if doc else "<no docstring>")

    def _user_names(self):
        hidden = {"session", "spark", "sc", "hc", "in_object", "out_object", "__builtins__"}
        import types
        return sorted(k for k, v in self.locals.items()
                      if not k.startswith("_") and k not in hidden and not isinstance(v, types.ModuleType))

    def _magic_time(self, stmt: str) -> None:
        import time
        t = time.perf_counter()
        try:
            val = eval(compile(stmt, "<magic>", "eval"), self.locals)
            is_expr = True
        except SyntaxError:
            exec(compile(stmt, "<magic>", "exec"), self.locals)
            is_expr, val = False, None
        el = time.perf_counter() - t
        print(f"Wall time: {_fmt_seconds(el)}")
        if is_expr and val is not None:
            print(repr(val))

    def _magic_timeit(self, arg: str) -> None:
        import shlex
        import timeit
        toks = shlex.split(arg)
        number, repeat = 0, 7
        while toks and toks[0] in ("-n", "-r") and len(toks) > 1:
            if toks[0] == "-n":
                number = int(toks[1])
            else:
                repeat = int(toks[1])
            toks = toks[2:]
        stmt = " ".join(toks)
        t = timeit.Timer(stmt, globals=self.locals)
        if number <= 0:
            number = t.autorange()[0]
        runs = [x / number for x in t.repeat(repeat=repeat, number=number)]
        mean = sum(runs) / len(runs)
        sd = (sum((x - mean) ** 2 for x in runs) / len(runs)) ** 0.5
        print(f"{_fmt_seconds(mean)} ± {_fmt_seconds(sd)} per loop (mean ± std. dev. of {repeat} runs, "
              f"{number} loops each)")

    def _magic_who(self, arg: str) -> None:
        names = self._user_names()
        print("  ".join(names) if names else "Interactive namespace is empty.")

    def _magic_whos(self, arg: str) -> None:
        names = self._user_names()
        if not names:
            print("Interactive namespace is empty.")
            return
        rows = [(n, type(self.locals[n]).__name__, repr(self.locals[n])[:60]) for n in names]
        w0 = max(8, max(len(r[0]) for r in rows))
        w1 = max(4, max(len(r[1]) for r in rows))
        print(f"{'Variable':<{w0}}   {'Type':<{w1}}   Data/Info")
        print("-" * (w0 + w1 + 16))
        for n, t, r in rows:
            print(f"{n:<{w0}}   {t:<{w1}}   {r}")

    def _magic_reset(self, arg: str) -> None:
        if "-f" not in arg.split():
            print("Use %reset -f to delete every user variable (session, in_object and out_object stay).")
            return
        for n in self._user_names():
            del self.locals[n]

    def _magic_history(self, arg: str) -> None:
        n = int(arg.lstrip("-n").strip() or 0) if arg else 0
        hist = [h for h in self.history if h.strip()][:-1]        # minus this %history line
        for h in hist[-n:] if n else hist:
            print(h)

    def _magic_run(self, path: str) -> None:
        with open(path, "rb") as f:
            src = f.read().decode("utf-8", errors="replace")
        self.locals.setdefault("__name__", "__main__")
        exec(compile(src, path, "exec"), self.locals)

    def _magic_pwd(self, arg: str) -> None:
        import os
        print(os.getcwd())

    def _magic_cd(self, arg: str) -> None:
        import os
        os.chdir(os.path.expanduser(arg or "~"))
        print(os.getcwd())

    def _magic_env(self, arg: str) -> None:
        import os
        if not arg:
            for k in sorted(os.environ):
                print(f"{k}={os.environ[k]}")
        elif "=" in arg:
            k, _, v = arg.partition("=")
            os.environ[k.strip()] = v.strip()
        else:
            print(os.environ.get(arg, ""))

    def _magic_lsmagic(self, arg: str) -> None:
        print("Available line magics:\n" + "  ".join("%" + m for m in self.MAGICS))

    def complete(self, text: str) -> list[str]:
        """Completions of the last token of ``text`` over the console namespace (names,
        attributes, keywords, builtins -- rlcompleter -- and the line magics)."""
        import rlcompleter
        m = re.search(r"[%\w.]*$", text)
        tok = m.group(0) if m else ""
        if tok.startswith("%"):
            return sorted("%" + k for k in self.MAGICS if k.startswith(tok[1:]))
        comp = rlcompleter.Completer(self.locals)
        out, i = [], 0
        while True:
            c = comp.complete(tok, i)
            if c is None:
                break
            if c not in out:
                out.append(c)
            i += 1
        return out

    def paste(self, source: str) -> bool:
        """Run pasted source line by line (reference pasteCode).  Unlike a bare REPL, a
        top-level line after an indented block first closes the block (as a file would run),
        and a trailing blank line closes a block left open."""
        for line in source.splitlines():
            if self.more and line and not line[0].isspace() and not _CONTINUES.match(line):
                self.push("")
            self.push(line)
        if self.more:
            self.push("")
        return self.more

    def history_prev(self) -> str:
        if not self.history:
            return ""
        self._hpos = max(0, self._hpos - 1)
        return self.history[self._hpos]

    def history_next(self) -> str:
        if not self.history:
            return ""
        self._hpos = min(len(self.history), self._hpos + 1)
        return self.history[self._hpos] if self._hpos < len(self.history) else ""


_CONTINUES = re.compile(r"(?:elif|else|except|finally|case)\b|[)\]}]")


def _fmt_seconds(t: float) -> str:
    for unit, scale in (("s", 1.0), ("ms", 1e-3), ("µs", 1e-6)):
        if t >= scale:
            return f"{t / scale:.3g} {unit}"
    return f"{t / 1e-9:.3g} ns"


class _Writer:
    def __init__(self, write):
        self.write = write

    def flush(self):
        pass


class _PerThreadStream:
    """Stand-in for ``sys.stdout`` / ``sys.stderr`` that sends a thread's writes to that
    thread's capture target (if one is set) and everyone else's to the stream it wraps.
    ``contextlib.redirect_stdout`` swaps the process-global stream, so a script running on
    a widget's worker thread would capture (and hide) the prints of every other thread
    for as long as it runs."""

    def __init__(self, base):
        self._base = base
        self._local = threading.local()

    def _target(self):
        t = getattr(self._local, "target", None)
        return self._base if t is None else t

    def write(self, data):
        return self._target().write(data)

    def flush(self):
        f = getattr(self._target(), "flush", None)
        if f is not None:
            f()

    def __getattr__(self, name):             # encoding, fileno, isatty, ... of the real stream
        return getattr(self._base, name)


_STREAM_LOCK = threading.Lock()


def _wrapped(name: str) -> "_PerThreadStream":
    with _STREAM_LOCK:
        cur = getattr(sys, name)
        if not isinstance(cur, _PerThreadStream):
            cur = _PerThreadStream(cur)
            setattr(sys, name, cur)
        return cur


@contextlib.contextmanager
def capture_output(target):
    """Send what THIS thread prints (stdout and stderr) to ``target`` (anything with a
    ``write``) for the duration; other threads' output is untouched."""
    streams = [_wrapped("stdout"), _wrapped("stderr")]
    prev = [getattr(st._local, "target", None) for st in streams]
    for st in streams:
        st._local.target = target
    try:
        yield target
    finally:
        for st, p in zip(streams, prev):
            st._local.target = p


def banner(session) -> str:
    v = getattr(session, "version", "?")
    return (f"Python {sys.version.split()[0]} on {sys.platform}\n"
            f"orange3-spark-amd {v}: session available as session / spark (sc, hc aliases); "
            f"in_object, out_object\n")
