"""Python Script widget parity with the reference PySpark Script console
(orangecontrib/spark/widgets/data/pyspark_script_console.py): interactive console over the
widget namespace (trash/OLDpyspark_script_console.py:125-286 semantics), import/save of
scripts (:368-392,441-461), syntax highlighting (:39-97) and auto-indent (:100-132)."""
import pytest

from orange3_spark_amd import Session, SessionConf
from orangecontrib.spark_amd.widgets.base import SharedSession
from orangecontrib.spark_amd.widgets.data.owscript import OWScript
from orangecontrib.spark_amd.widgets.script_support import (ScriptConsole, backspace_width, highlight_spans,
                                                            indent_after)


@pytest.fixture(scope="module")
def session():
    s = Session(SessionConf().set("o3s.device", "cpu"))
    SharedSession._session = s
    yield s
    SharedSession._session = None


def test_console_lines_share_state_and_read_back_out_object(session):
    w = OWScript()
    w.set_in_object(session.range(0, 7))
    assert not w.console_push("n = in_object.count()")
    assert not w.console_push("out_object = n * 3")
    assert w.out_object == 21
    assert "Python" in w.console_output and "session available" in w.console_output
    # a block stays open until a blank line, then runs
    assert w.console_push("def twice(v):")
    assert w.console_push("    return 2 * v")
    assert not w.console_push("")
    w.console_push("print(twice(out_object))")
    assert "42" in w.console_output
    # errors are printed, the console keeps going
    w.console_push("1 / 0")
    assert "ZeroDivisionError" in w.console_output
    w.console_push("out_object = twice(5)")
    assert w.out_object == 10
    # the script sees what the console defined (one namespace)
    w.scriptText = "out_object = twice(n)"
    assert w.commit() == 14 and w.sent["out_object"] == 14
    # history walks back over the typed lines
    assert w.console_history(-1) == "out_object = twice(5)"
    assert w.console_history(-1) == "1 / 0"
    assert w.console_history(+1) == "out_object = twice(5)"


def test_console_paste_runs_multiline_source(session):
    w = OWScript()
    w.console_paste("total = 0\nfor i in range(4):\n    total += i\nout_object = total")
    assert w.out_object == 6
    assert "... " in w.console_output


def test_import_and_save_scripts(tmp_path, session):
    w = OWScript()
    p = tmp_path / "etl.py"
    p.write_bytes("out_object = 'ünï'\n".encode("utf-8"))
    i = w.import_script(str(p))
    assert w.libraryListSource[i]["name"] == "etl.py" and w.current_script() == "out_object = 'ünï'\n"
    assert w.commit() == "ünï"
    w.scriptText = "out_object = 5\n"                     # unsaved editor edits are what gets saved
    out = w.save_script(str(tmp_path / "saved"))
    assert out.endswith("saved.py") and open(out, encoding="utf-8").read() == "out_object = 5\n"
    assert w.libraryListSource[i]["filename"].endswith("saved.py")
    w.update_script(i, "out_object = 6\n")
    assert w.save_script() == out and open(out).read() == "out_object = 6\n"   # default: its file
    w2 = OWScript()
    w2.import_script(out)
    assert w2.commit() == 6
    with pytest.raises(ValueError):
        OWScript().save_script()                          # no file name known


def test_auto_indent_rules_match_reference_editor():
    assert indent_after("for x in y:") == 4
    assert indent_after("    if a:") == 8
    assert indent_after("        pass") == 4
    assert indent_after("        return x") == 4
    assert indent_after("    y = 1") == 4
    assert indent_after("# comment:") == 0
    assert backspace_width("        ") == 4 and backspace_width("  ") == 2 and backspace_width("  x") == 1


def _fmt_at(spans, i):
    got = None
    for a, n, f in spans:
        if a <= i < a + n:
            got = f                                       # later spans override
    return got


def test_highlighter_spans():
    line = "def load(path):  # read 'x'"
    spans, st = highlight_spans(line)
    assert st == 0
    assert _fmt_at(spans, 0) == "keyword" and _fmt_at(spans, 4) == "def"
    assert _fmt_at(spans, line.index("#")) == "comment" and _fmt_at(spans, line.index("'x'")) == "comment"
    spans, _ = highlight_spans("s = 'a # b' + 3")
    assert _fmt_at(spans, 5) == "string" and _fmt_at(spans, 7) == "string" and _fmt_at(spans, 14) == "number"
    spans, _ = highlight_spans("@decorator")
    assert _fmt_at(spans, 1) == "decorator"
    # triple-quoted strings carry over lines through the block state
    spans, st = highlight_spans('doc = """start')
    assert st == 2 and _fmt_at(spans, 8) == "string"
    spans, st = highlight_spans("middle if else", st)
    assert st == 2 and spans == [(0, 14, "string")]
    spans, st = highlight_spans('end""" + x', st)
    assert st == 0 and _fmt_at(spans, 2) == "string" and _fmt_at(spans, 8) is None


def test_console_class_standalone():
    out = []
    c = ScriptConsole({}, out.append)
    c.push("a = [1,")
    assert c.more and c.prompt == "... "
    c.push("2]")
    c.push("print(sum(a))")
    assert "3\n" in "".join(out)


def test_console_ipython_conveniences(session, tmp_path):
    """The reference's console is an embedded IPython kernel (pyspark_script_console.py:
    20-29,331); without IPython the console still takes line magics, ``obj?`` help, ``!cmd``
    and Tab completion over the widget namespace."""
    w = OWScript()
    w.console_push("%time total = sum(range(1000))")
    assert "Wall time:" in w.console_output and w.namespace["total"] == 499500
    w.console_push("%timeit -n 5 -r 2 sum(range(100))")
    assert "per loop (mean ± std. dev. of 2 runs, 5 loops each)" in w.console_output
    w.console_push("%who")
    assert "total" in w.console_output.splitlines()[-1]
    w.console_push("%whos")
    assert "Variable" in w.console_output and "int" in w.console_output
    w.console_push("def twice(v):")
    w.console_push("    '''Double v.'''")
    w.console_push("    return 2 * v")
    w.console_push("")
    w.console_push("twice?")
    assert "Signature: twice(v)" in w.console_output and "Double v." in w.console_output
    w.console_push("twice??")
    assert "return 2 * v" in w.console_output
    w.console_push("nothing_here?")
    assert "Object `nothing_here` not found" in w.console_output
    w.console_push("!echo shell-says-hi")
    assert "shell-says-hi" in w.console_output
    w.console_push("%nosuchmagic")
    assert "UsageError: Line magic function `%nosuchmagic` not found." in w.console_output
    p = tmp_path / "snippet.py"
    p.write_text("out_object = twice(total)\n")
    w.console_push(f"%run {p}")
    assert w.out_object == 999000
    w.console_push("%history -n 2")
    assert w.console_output.rstrip().endswith(f"%run {p}")
    # completion: names, attributes, magics
    assert "twice(" in w.console_complete("print(twi")
    assert any(c.startswith("total.") for c in w.console_complete("total.bit"))
    assert w.console_complete("%tim") == ["%time", "%timeit"]
    # session objects survive %reset -f; user names do not
    w.console_push("%reset -f")
    assert "total" not in w.namespace and "twice" not in w.namespace
    assert w.namespace["session"] is session
    # plain Python still flows through (a block is never taken for a magic)
    assert w.console_push("for i in range(2):")
    assert w.console_push("    out_object = i")
    assert not w.console_push("")
    assert w.out_object == 1


def test_console_tab_completion_text():
    from orangecontrib.spark_amd.widgets.custom_views import complete_line
    assert complete_line("x = ran", ["range("]) == ("x = range(", "")
    text, listing = complete_line("%ti", ["%time", "%timeit"])
    assert text == "%time" and listing == "%time  %timeit\n"
    assert complete_line("zz", []) == ("zz", "")
