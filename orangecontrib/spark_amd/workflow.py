"""Headless workflow runner: load/save Orange ``.ows`` schemes and run them on the
compat signal manager.

Reference workflows (e.g. orangecontrib/spark/tutorials/spark_ml.ows, nodes :3-12, links
:13-20, node_properties :39-57) name the reference's widget classes; they are mapped to
this add-on's widgets by ``REFERENCE_WIDGETS``.  Node properties stored as ``literal`` are
parsed with ``ast.literal_eval``; ``pickle`` properties are NEVER unpickled (they only hold
Qt window geometry in the reference tutorial) and are skipped with a warning.
"""
from __future__ import annotations

import ast
import importlib
import logging
import xml.etree.ElementTree as ET
from dataclasses import dataclass, field

from .widgets.compat import SignalManager, Widget

log = logging.getLogger(__name__)

_P = "orangecontrib.spark_amd.widgets"
REFERENCE_WIDGETS = {
    "orangecontrib.spark.widgets.data.spark_context.OWSparkContext": f"{_P}.data.owcontext.OWSessionContext",
    "orangecontrib.spark.widgets.data.spark_table.OWSparkSQLTableContext": f"{_P}.data.owtable.OWCatalogTable",
    "orangecontrib.spark.widgets.data.spark_sql_dataframe.OWSparkDataFrame": f"{_P}.data.owsql.OWSQLDataFrame",
    "orangecontrib.spark.widgets.data.odbc_table.OWodbcTable": f"{_P}.data.owdatabase.OWDatabase",
    "orangecontrib.spark.widgets.data.pyspark_script_console.OWPySparkScript": f"{_P}.data.owscript.OWScript",
    "orangecontrib.spark.widgets.data.spark_fill.OWSparkFillNa": f"{_P}.data.owfillna.OWFillNa",
    "orangecontrib.spark.widgets.data.spark_sample.OWSparkDFSample": f"{_P}.data.owsample.OWSample",
    "orangecontrib.spark.widgets.data.spark_df_cache.OWSparkMLMOdel": f"{_P}.data.owcache.OWCacheDataFrame",
    "orangecontrib.spark.widgets.data.spark_from_orange.OWSparkFromOrange": f"{_P}.data.owfromorange.OWFromOrange",
    "orangecontrib.spark.widgets.data.spark_from_pandas.OWSparkToPandas": f"{_P}.data.owfrompandas.OWFromPandas",
    "orangecontrib.spark.widgets.data.spark_to_orange.OWSparkToOrange": f"{_P}.data.owtoorange.OWToOrange",
    "orangecontrib.spark.widgets.data.spark_to_pandas.OWSparkToPandas": f"{_P}.data.owtopandas.OWToPandas",
    "orangecontrib.spark.widgets.data.pandas_to_orange.OWPandasToOrange":
        f"{_P}.data.owpandastoorange.OWPandasToOrange",
    "orangecontrib.spark.widgets.data.orange_to_pandas.OWOrangeToPandas":
        f"{_P}.data.oworangetopandas.OWOrangeToPandas",
    "orangecontrib.spark.widgets.ml.spark_ml_classification.OWSparkMLClassification":
        f"{_P}.ml.owclassification.OWClassification",
    "orangecontrib.spark.widgets.ml.spark_ml_clustering.OWSparkMLClustering": f"{_P}.ml.owclustering.OWClustering",
    "orangecontrib.spark.widgets.ml.spark_ml_regression.OWSparkMLRegression": f"{_P}.ml.owregression.OWRegression",
    "orangecontrib.spark.widgets.ml.spark_ml_recommendation.OWSparkMLRecommendation":
        f"{_P}.ml.owrecommendation.OWRecommendation",
    "orangecontrib.spark.widgets.ml.spark_ml_dataset.OWSparkMLDatasetBuilder":
        f"{_P}.ml.owdatasetbuilder.OWDatasetBuilder",
    "orangecontrib.spark.widgets.ml.spark_ml_feature.OWSparkMLFeature": f"{_P}.ml.owfeature.OWFeature",
    "orangecontrib.spark.widgets.ml.spark_ml_model.OWSparkMLMOdel": f"{_P}.ml.owmodeltransformer.OWModelTransformer",
    "orangecontrib.spark.widgets.ml.spark_ml_evaluation.OWSparkMLEvaluator": f"{_P}.ml.owevaluation.OWEvaluation",
}


def _plain(v):
    """Literal-safe copy (OrderedDict -> dict, tuples kept) for ``ast.literal_eval`` round trips."""
    if isinstance(v, dict):
        return {k: _plain(x) for k, x in v.items()}
    if isinstance(v, list):
        return [_plain(x) for x in v]
    if isinstance(v, tuple):
        return tuple(_plain(x) for x in v)
    return v


def resolve(qualified_name: str) -> type:
    """Headless widget class of a workflow node.  Accepts the reference's names
    (REFERENCE_WIDGETS), the Qt view names Orange registers (``...OWSessionContextView``:
    the view's ``core_class``, or the name without ``View`` when Orange is absent and no
    view was generated) and headless class names."""
    qn = REFERENCE_WIDGETS.get(qualified_name, qualified_name)
    mod, _, cls = qn.rpartition(".")
    m = importlib.import_module(mod)
    obj = getattr(m, cls, None)
    if obj is None and cls.endswith("View"):
        obj = getattr(m, cls[:-4], None)
    if obj is None:
        raise ImportError(f"cannot resolve widget {qualified_name}")
    return getattr(obj, "core_class", obj)


@dataclass
class Node:
    id: str
    qualified_name: str
    title: str
    properties: dict = field(default_factory=dict)
    widget: Widget | None = None
    position: tuple = (0.0, 0.0)


@dataclass
class Link:
    source: str
    source_channel: str
    sink: str
    sink_channel: str
    enabled: bool = True


class Workflow:
    def __init__(self, title: str = "", description: str = ""):
        self.title, self.description = title, description
        self.nodes: dict[str, Node] = {}
        self.links: list[Link] = []
        # canvas annotations: ("text", rect(x, y, w, h), text, font_size) or
        # ("arrow", start(x, y), end(x, y), fill colour)
        self.annotations: list[tuple] = []
        self.manager = SignalManager()

    # -- construction ------------------------------------------------------------
    def add_node(self, qualified_name, title=None, properties=None, node_id=None, position=None) -> Node:
        nid = str(node_id if node_id is not None else len(self.nodes))
        n = Node(nid, qualified_name, title or qualified_name.rsplit(".", 1)[-1], dict(properties or {}))
        if position is not None:
            n.position = tuple(float(v) for v in position)
        self.nodes[nid] = n
        return n

    def add_text(self, rect, text, font_size=16):
        self.annotations.append(("text", tuple(float(v) for v in rect), str(text), int(font_size)))

    def add_arrow(self, start, end, fill="#C1272D"):
        self.annotations.append(("arrow", tuple(float(v) for v in start), tuple(float(v) for v in end), str(fill)))

    def add_link(self, source, source_channel, sink, sink_channel, enabled=True):
        self.links.append(Link(str(source), source_channel, str(sink), sink_channel, enabled))

    @classmethod
    def load(cls, path: str) -> "Workflow":
        root = ET.parse(path).getroot()
        wf = cls(root.get("title", ""), root.get("description", ""))
        for n in root.iter("node"):
            pos = None
            try:
                pos = ast.literal_eval(n.get("position") or "None")
            except (ValueError, SyntaxError):
                pass
            wf.add_node(n.get("qualified_name"), n.get("title"), node_id=n.get("id"),
                        position=pos if isinstance(pos, tuple) and len(pos) == 2 else None)
        for a in root.iter("text"):
            try:
                wf.add_text(ast.literal_eval(a.get("rect")), a.text or "", int(a.get("font-size", "16")))
            except (ValueError, SyntaxError, TypeError):
                pass
        for a in root.iter("arrow"):
            try:
                wf.add_arrow(ast.literal_eval(a.get("start")), ast.literal_eval(a.get("end")), a.get("fill", "#C1272D"))
            except (ValueError, SyntaxError, TypeError):
                pass
        for ln in root.iter("link"):
            wf.add_link(ln.get("source_node_id"), ln.get("source_channel"), ln.get("sink_node_id"),
                        ln.get("sink_channel"), ln.get("enabled", "true") == "true")
        for p in root.iter("properties"):
            nid, fmt = p.get("node_id"), p.get("format")
            if fmt == "literal":
                try:
                    props = ast.literal_eval((p.text or "").strip())
                except (ValueError, SyntaxError):
                    props = {}
                wf.nodes[nid].properties = {k: v for k, v in props.items() if k != "savedWidgetGeometry"}
            else:
                log.warning("node %s: skipping %s-format properties (never unpickled)", nid, fmt)
        return wf

    def save(self, path: str) -> None:
        root = ET.Element("scheme", {"version": "2.0", "title": self.title, "description": self.description})
        nodes = ET.SubElement(root, "nodes")
        for n in self.nodes.values():
            ET.SubElement(nodes, "node", {"id": n.id, "name": n.title, "qualified_name": n.qualified_name,
                                          "project_name": "Orange3-Spark-AMD", "title": n.title, "version": "",
                                          "position": repr(tuple(n.position))})
        links = ET.SubElement(root, "links")
        for i, ln in enumerate(self.links):
            ET.SubElement(links, "link", {"id": str(i), "source_node_id": ln.source, "sink_node_id": ln.sink,
                                          "source_channel": ln.source_channel, "sink_channel": ln.sink_channel,
                                          "enabled": "true" if ln.enabled else "false"})
        ann = ET.SubElement(root, "annotations")
        for i, a in enumerate(self.annotations):
            if a[0] == "text":
                e = ET.SubElement(ann, "text", {"id": str(i), "rect": repr(a[1]), "font-family": "Helvetica",
                                                "font-size": str(a[3])})
                e.text = a[2]
            else:
                ET.SubElement(ann, "arrow", {"id": str(i), "start": repr(a[1]), "end": repr(a[2]), "fill": a[3]})
        props = ET.SubElement(root, "node_properties")
        for n in self.nodes.values():
            d = n.widget.settings_dict() if n.widget is not None else n.properties
            e = ET.SubElement(props, "properties", {"node_id": n.id, "format": "literal"})
            e.text = repr(_plain(d))
        ET.ElementTree(root).write(path, encoding="utf-8", xml_declaration=True)

    # -- execution ---------------------------------------------------------------
    def instantiate(self) -> "Workflow":
        for n in self.nodes.values():
            cls = resolve(n.qualified_name)
            w = cls()
            w.apply_settings(n.properties)
            n.widget = self.manager.add(w)
        for ln in self.links:
            if ln.enabled:
                src, dst = self.nodes[ln.source].widget, self.nodes[ln.sink].widget
                self.manager.link(src, ln.source_channel, dst, ln.sink_channel)
        return self

    def widget(self, key) -> Widget:
        if key in self.nodes:
            return self.nodes[key].widget
        for n in self.nodes.values():
            if n.title == key:
                return n.widget
        raise KeyError(key)
