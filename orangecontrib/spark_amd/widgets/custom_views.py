"""Hand-written canvas controls for the widgets whose reference UI is not a parameter form.

``views.qt_view`` builds generic editors (line edits / check boxes / reflective combo
boxes); the three widgets below need list and editor controls to be usable from the Orange
canvas, as in the reference:

* Dataset Builder -- available / features / label / meta column lists with a filter and
  move / reorder buttons (reference widgets/ml/spark_ml_dataset.py:292-593, commit
  :569-582);
* Hive Table -- database and table combo boxes filled from the catalog
  (reference widgets/data/spark_table.py:40-70);
* Python Script -- script library list with add / remove / update, a multi-line editor
  and a console pane showing the script's output (reference
  widgets/data/pyspark_script_console.py:206-466).

A builder receives the Qt view (``view.core`` is the headless widget) and the
``orange`` namespace (``gui`` helpers and the ``qt`` widgets module); it returns the
settings its controls cover (no generic editor is made for those) and a ``refresh``
callable the view runs after every input and action.  Only plain QtWidgets calls are
used (QListWidget, QComboBox, QPlainTextEdit, QLineEdit, QPushButton, QTextBrowser).
"""
from __future__ import annotations


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
def build_script(view, orange):
    qt, gui, core = orange.qt, orange.gui, view.core
    lib_box = gui.widgetBox(view.controlArea, "Library")
    ll = lib_box.layout()
    library = _list(qt, multi=False)
    ll.addWidget(library)
    edit_box = gui.widgetBox(view.controlArea, "Script")
    el = edit_box.layout()
    editor = qt.QPlainTextEdit()
    el.addWidget(editor)
    console = qt.QTextBrowser()
    view.mainArea.layout().addWidget(console) if getattr(view, "mainArea", None) is not None else el.addWidget(console)
    view.script_controls = {"library": library, "editor": editor, "console": console}
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
    library.currentRowChanged.connect(selected)
    editor.textChanged.connect(edited)
    _button(qt, ll, "+", add)
    _button(qt, ll, "-", remove)
    _button(qt, ll, "Update", update)
    _button(qt, el, "Clear console", clear_console)
    return {"libraryListSource", "currentScriptIndex", "scriptText"}, refresh


BUILDERS = {"OWDatasetBuilder": build_dataset_builder, "OWCatalogTable": build_catalog_table,
            "OWScript": build_script}
