"""Regenerate orangecontrib/spark_amd/tutorials/spark_ml.ows (same graph as the
reference tutorial, orangecontrib/spark/tutorials/spark_ml.ows:3-20, with this add-on's
widgets and literal-format settings).  Nodes name the Qt view classes (``...View``) --
the classes Orange's widget discovery registers -- so the canvas can open the file; the
headless runner maps them to their headless cores (workflow.resolve)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orangecontrib.spark_amd.workflow import Workflow  # noqa: E402

P = "orangecontrib.spark_amd.widgets"
wf = Workflow("Spark ML tutorial (MI355X)", "Context -> catalog tables -> Dataset Builder -> Classification -> "
              "Model Transformer -> Evaluation. Create the session first.")
wf.add_node(f"{P}.data.owcontext.OWSessionContextView", "Context", node_id=0)
wf.add_node(f"{P}.data.owtable.OWCatalogTableView", "Training data", {"database": "default", "table": "train"}, 1)
wf.add_node(f"{P}.ml.owdatasetbuilder.OWDatasetBuilderView", "Dataset Builder", node_id=2)
wf.add_node(f"{P}.ml.owclassification.OWClassificationView", "Classification", node_id=3)
wf.add_node(f"{P}.ml.owmodeltransformer.OWModelTransformerView", "Model Transformer", node_id=4)
wf.add_node(f"{P}.data.owtable.OWCatalogTableView", "Testing Data", {"database": "default", "table": "test"}, 5)
wf.add_node(f"{P}.ml.owdatasetbuilder.OWDatasetBuilderView", "Dataset Builder (1)", node_id=6)
wf.add_node(f"{P}.ml.owevaluation.OWEvaluationView", "Evaluation", node_id=7)
wf.add_link(2, "DataFrame", 3, "DataFrame")
wf.add_link(3, "Model", 4, "Model")
wf.add_link(1, "DataFrame", 2, "DataFrame")
wf.add_link(5, "DataFrame", 6, "DataFrame")
wf.add_link(6, "DataFrame", 4, "DataFrame")
wf.add_link(4, "DataFrame", 7, "DataFrame")
out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "orangecontrib", "spark_amd",
                   "tutorials", "spark_ml.ows")
wf.save(out)
print(out)
