"""Hand-written canvas controls for the widgets whose reference UI is not a parameter form.

``views.qt_view`` builds generic editors (line edits / check boxes / reflective combo
boxes); the three widgets below need list and editor controls to be usable from the Orange
canvas, as in the reference:

* Dataset Builder -- available / features / label / meta column lists with a filter and
  move / reorder buttons (reference widgets/ml/spark_ml_dataset.py:292-593, commit
  :569-582);
* Hive Table -- database and table combo boxes filled from the catalog
  (reference widgets/data/spark_table.py:40-70);
* Python Script -- script library list with add / remove / update / import from file /
  save to file, an auto-indenting editor with a Python syntax highlighter, and a console
  pane with an input line running statements in the script's namespace (reference
  widgets/data/pyspark_script_console.py:39-132,206-466).

A builder receives the Qt view (``view.core`` is the headless widget) and the
``orange`` namespace (``gui`` helpers and the ``qt`` widgets module); it returns the
settings its controls cover (no generic editor is made for those) and a ``refresh``
callable the view runs after every input and action.  Only plain QtWidgets calls are
used (QListWidget, QComboBox, QPlainTextEdit, QLineEdit, QPushButton, QTextBrowser,
QFileDialog), plus QtGui.QSyntaxHighlighter / QtCore key codes for the script editor when
the namespace provides ``qtgui`` / ``qtcore``.
"""
from __future__ import annotations

import re
import os


def _list(qt, multi=True):
    w = qt.QListWidget()
    if multi:
        mode = getattr(getattr(qt, "QAbstractItemView", None), "ExtendedSelection", None)
        if mode is not None:
            w.setSelectionMode(mode)
    return w


def _selected(w) -> list:
    return [it.text() for it in w.selectedItems()]


def _fill(w, items):
    w.clear()
    w.addItems([str(x) for x in items])


def _button(qt, lay, text, fn):
    b = qt.QPushButton(text)
    b.clicked.connect(lambda *_: fn())
    lay.addWidget(b)
    return b


# ------------------------------------------------------------------------------ builder
def build_dataset_builder(view, orange):
    qt, gui, core = orange.qt, orange.gui, view.core
    box = gui.widgetBox(view.controlArea, "Columns")
    lay = box.layout()
    filt = qt.QLineEdit()
    filt.setPlaceholderText("Filter available columns...")
    lay.addWidget(qt.QLabel("Available"))
    lay.addWidget(filt)
    avail = _list(qt)
    lay.addWidget(avail)
    moves = gui.widgetBox(view.controlArea, "Assign")
    ml = moves.layout()
    lay2 = gui.widgetBox(view.controlArea, "Roles").layout()
    lay2.addWidget(qt.QLabel("Features"))
    feats = _list(qt)
    lay2.addWidget(feats)
    lay2.addWidget(qt.QLabel("Label (at most one)"))
    label = _list(qt, multi=False)
    lay2.addWidget(label)
    lay2.addWidget(qt.QLabel("Meta"))
    metas = _list(qt)
    lay2.addWidget(metas)
    view.builder_lists = {"available": avail, "features": feats, "label": label, "metas": metas, "filter": filt}

    def refresh():
        _fill(avail, core.filtered_available(filt.text()))
        _fill(feats, core.used_attrs)
        _fill(label, core.class_attrs)
        _fill(metas, core.meta_attrs)

    def to_features():
        core.set_features(_selected(avail))
        refresh()

    def to_label():
        sel = _selected(avail) or _selected(feats) or _selected(metas)
        if sel:
            core.set_label(sel[0])
        refresh()

    def to_metas():
        core.set_metas(_selected(avail) + _selected(feats))
        refresh()

    def back():
        core.move_to_available(_selected(feats) + _selected(label) + _selected(metas))
        refresh()

    def up():
        for name in _selected(feats):
            core.move_feature(name, -1)
        refresh()

    def down():
        for name in reversed(_selected(feats)):
            core.move_feature(name, +1)
        refresh()

    def reset():
        core.reset()
        refresh()
    _button(qt, ml, "Features >", to_features)
    _button(qt, ml, "Label >", to_label)
    _button(qt, ml, "Meta >", to_metas)
    _button(qt, ml, "< Available", back)
    _button(qt, ml, "Up", up)
    _button(qt, ml, "Down", down)
    _button(qt, ml, "Reset", reset)
    filt.textChanged.connect(lambda *_: refresh())
    return {"domain_role_hints"}, refresh


# ------------------------------------------------------------------------------ table
def build_catalog_table(view, orange):
    qt, gui, core = orange.qt, orange.gui, view.core
    box = gui.widgetBox(view.controlArea, "Catalog")
    lay = box.layout()
    lay.addWidget(qt.QLabel("Database"))
    dbs = qt.QComboBox()
    lay.addWidget(dbs)
    lay.addWidget(qt.QLabel("Table"))
    tables = qt.QComboBox()
    lay.addWidget(tables)
    view.table_controls = {"databases": dbs, "tables": tables}
    state = {"busy": False}

    def refresh():
        state["busy"] = True
        try:
            _fill(dbs, core.databases)
            dbs.setCurrentText(str(core.database))
            _fill(tables, core.tables)
            if core.table in core.tables:
                tables.setCurrentText(str(core.table))
            elif core.tables:
                core.table = core.tables[0]
                tables.setCurrentText(str(core.table))
        finally:
            state["busy"] = False

    def db_changed(text):
        if state["busy"] or not text:
            return
        core.refresh_tables(text)
        view.database = core.database
        refresh()

    def table_changed(text):
        if state["busy"] or not text:
            return
        core.table = text
        view.table = text

    def reload():
        core.refresh()
        refresh()
    dbs.currentTextChanged.connect(db_changed)
    tables.currentTextChanged.connect(table_changed)
    _button(qt, lay, "Refresh", reload)
    return {"database", "table"}, refresh


# ------------------------------------------------------------------------------ script
def _script_editor(qt, qtcore):
    """QPlainTextEdit with the reference's auto-indent keys (PythonScriptEditor,
    pyspark_script_console.py:100-132): Return keeps the indent (+4 after ':', -4 after
    pass/return), Tab inserts 4 spaces, Backspace in leading blanks removes one step."""
    if qtcore is None:
        return qt.QPlainTextEdit()
    from .script_support import INDENT, backspace_width, indent_after
    K = qtcore.Qt

    class ScriptEditor(qt.QPlainTextEdit):
        def _line(self):
            cur = self.textCursor()
            return cur, cur.block().text()[:cur.positionInBlock()]

        def keyPressEvent(self, ev):
            k = ev.key()
            if k in (K.Key_Return, K.Key_Enter):
                _, line = self._line()
                super().keyPressEvent(ev)
                self.insertPlainText(" " * indent_after(line))
            elif k == K.Key_Tab:
                self.insertPlainText(" " * INDENT)
            elif k == K.Key_Backspace:
                cur, line = self._line()
                if cur.hasSelection():
                    super().keyPressEvent(ev)
                else:
                    for _ in range(backspace_width(line)):
                        cur.deletePreviousChar()
            else:
                super().keyPressEvent(ev)
    return ScriptEditor()


def _highlighter(qtgui, document):
    """QSyntaxHighlighter over script_support.highlight_spans (ref PythonSyntaxHighlighter,
    pyspark_script_console.py:39-97)."""
    if qtgui is None or document is None:
        return None
    from .script_support import FORMATS, highlight_spans

    class PythonHighlighter(qtgui.QSyntaxHighlighter):
        def __init__(self, doc):
            super().__init__(doc)
            self._fmt = {}
            for name, (color, bold) in FORMATS.items():
                f = qtgui.QTextCharFormat()
                f.setForeground(qtgui.QColor(color.lower()))
                if bold:
                    f.setFontWeight(qtgui.QFont.Bold)
                self._fmt[name] = f

        def highlightBlock(self, text):
            spans, state = highlight_spans(str(text), max(0, self.previousBlockState()))
            for start, n, fmt in spans:
                self.setFormat(start, n, self._fmt[fmt])
            self.setCurrentBlockState(state)
    return PythonHighlighter(document)


def complete_line(text: str, matches: list) -> tuple:
    """Tab in the console input: (new text, listing) -- one match replaces the last token,
    several extend it by their common prefix and are listed in the console."""
    import os
    m = re.search(r"[%\w.]*$", text)
    tok = m.group(0) if m else ""
    if not matches:
        return text, ""
    if len(matches) == 1:
        return text[:len(text) - len(tok)] + matches[0], ""
    common = os.path.commonprefix(matches)
    return text[:len(text) - len(tok)] + (common if len(common) > len(tok) else tok), "  ".join(matches) + "\n"


def _console_input(qt, qtcore, core, refresh):
    """One-line console input: Return runs the line, Up/Down walk the history, Tab completes."""
    if qtcore is None:
        line = qt.QLineEdit()
    else:
        K = qtcore.Qt

        class ConsoleLine(qt.QLineEdit):
            def event(self, ev):        # Tab would move the focus before keyPressEvent sees it
                if getattr(ev, "type", lambda: None)() == qtcore.QEvent.KeyPress and ev.key() == K.Key_Tab:
                    text, listing = complete_line(self.text(), core.console_complete(self.text()))
                    self.setText(text)
                    if listing:
                        core.console_output += listing
                        refresh()
                    return True
                return super().event(ev)

            def keyPressEvent(self, ev):
                if ev.key() == K.Key_Up:
                    self.setText(core.console_history(-1))
                elif ev.key() == K.Key_Down:
                    self.setText(core.console_history(+1))
                else:
                    super().keyPressEvent(ev)
        line = ConsoleLine()
    line.setPlaceholderText(">>> run a line in the script namespace")

    def run():
        core.console_push(line.text())
        line.setText("")
        refresh()
    line.returnPressed.connect(run)
    return line


def build_script(view, orange):
    qt, gui, core = orange.qt, orange.gui, view.core
    qtgui, qtcore = getattr(orange, "qtgui", None), getattr(orange, "qtcore", None)
    lib_box = gui.widgetBox(view.controlArea, "Library")
    ll = lib_box.layout()
    library = _list(qt, multi=False)
    ll.addWidget(library)
    edit_box = gui.widgetBox(view.controlArea, "Script")
    el = edit_box.layout()
    editor = _script_editor(qt, qtcore)
    highlighter = _highlighter(qtgui, editor.document() if hasattr(editor, "document") else None)
    el.addWidget(editor)
    console = qt.QTextBrowser()
    main = view.mainArea.layout() if getattr(view, "mainArea", None) is not None else el
    main.addWidget(console)
    state = {"busy": False}

    def refresh():
        state["busy"] = True
        try:
            _fill(library, [s["name"] for s in core.libraryListSource])
            if core.libraryListSource:
                library.setCurrentRow(core.currentScriptIndex)
            editor.setPlainText(core.current_script())
            console.setPlainText(core.console_output)
        finally:
            state["busy"] = False

    entry = _console_input(qt, qtcore, core, refresh)
    main.addWidget(entry)
    view.script_controls = {"library": library, "editor": editor, "console": console, "console_input": entry,
                            "highlighter": highlighter}

    def selected(row):
        if state["busy"] or row is None or row < 0:
            return
        core.select_script(row)
        view.currentScriptIndex = core.currentScriptIndex
        view.scriptText = core.scriptText
        refresh()

    def edited(*_):
        if state["busy"]:
            return
        core.scriptText = editor.toPlainText()
        view.scriptText = core.scriptText

    def add():
        core.add_script(f"Script {len(core.libraryListSource) + 1}", editor.toPlainText())
        refresh()

    def remove():
        if core.libraryListSource:
            core.remove_script(core.currentScriptIndex)
        refresh()

    def update():
        core.update_script(core.currentScriptIndex, editor.toPlainText())
        refresh()

    def clear_console():
        core.console_output = ""
        refresh()

    def _name(got):
        return got[0] if isinstance(got, tuple) else got

    def import_file():
        name = _name(qt.QFileDialog.getOpenFileName(view, "Open Python Script", os.path.expanduser("~/"),
                                                    "Python files (*.py);;All files (*.*)"))
        if name:
            core.import_script(str(name))
            view.currentScriptIndex = core.currentScriptIndex
            refresh()

    def save_file():
        cur = core.libraryListSource[core.currentScriptIndex] if core.libraryListSource else {}
        name = _name(qt.QFileDialog.getSaveFileName(view, "Save Python Script",
                                                    cur.get("filename") or os.path.expanduser("~/"),
                                                    "Python files (*.py);;All files (*.*)"))
        if name:
            core.save_script(str(name))
            refresh()
    library.currentRowChanged.connect(selected)
    editor.textChanged.connect(edited)
    _button(qt, ll, "+", add)
    _button(qt, ll, "-", remove)
    _button(qt, ll, "Update", update)
    _button(qt, ll, "Import a script from a file", import_file)
    _button(qt, ll, "Save selected script to a file", save_file)
    _button(qt, el, "Clear console", clear_console)
    return {"libraryListSource", "currentScriptIndex", "scriptText"}, refresh


BUILDERS = {"OWDatasetBuilder": build_dataset_builder, "OWCatalogTable": build_catalog_table,
            "OWScript": build_script}
