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
