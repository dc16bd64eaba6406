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
wf = Workflow("Spark ML tutorial (MI355X)",
              "This tutorial shows a basic flow to work with the ML widgets.\n\nThe session (Context) is shared "
              "by all widgets and should be created first; spark.executor.instances=auto uses every MI355X.")
# node positions and annotations follow the reference layout (spark_ml.ows:4-11,22-37)
wf.add_node(f"{P}.data.owcontext.OWSessionContextView", "Context", node_id=0, position=(41, 97))
wf.add_node(f"{P}.data.owtable.OWCatalogTableView", "Training data", {"database": "default", "table": "train"}, 1,
            position=(41, 247))
wf.add_node(f"{P}.ml.owdatasetbuilder.OWDatasetBuilderView", "Dataset Builder", node_id=2, position=(191, 247))
wf.add_node(f"{P}.ml.owclassification.OWClassificationView", "Classification", node_id=3, position=(341, 247))
wf.add_node(f"{P}.ml.owmodeltransformer.OWModelTransformerView", "Model Transformer", node_id=4,
            position=(491, 397))
wf.add_node(f"{P}.data.owtable.OWCatalogTableView", "Testing Data", {"database": "default", "table": "test"}, 5,
            position=(41, 397))
wf.add_node(f"{P}.ml.owdatasetbuilder.OWDatasetBuilderView", "Dataset Builder (1)", node_id=6, position=(191, 397))
wf.add_node(f"{P}.ml.owevaluation.OWEvaluationView", "Evaluation", node_id=7, position=(641, 397))
wf.add_arrow((184, 34), (77, 81), "#C1272D")
wf.add_text((190, 15, 245, 31), "First, create the session (Context)", 18)
wf.add_arrow((180, 143), (77, 213), "#C1272D")
wf.add_text((179, 117, 436, 21), "DataFrame from a catalog (Hive) table", 20)
wf.add_arrow((337, 568), (234, 462), "#39B54A")
wf.add_arrow((337, 566), (222, 309), "#39B54A")
wf.add_text((334, 559, 309, 56), "Select columns as the classification features and the label column", 18)
wf.add_arrow((529, 193), (377, 233), "#1F9CDF")
wf.add_text((535, 165, 269, 50), "Select a classification algorithm\nand obtain a fitted model", 16)
wf.add_text((539, 234, 256, 50), "Apply the fitted model to the testing dataset", 16)
wf.add_arrow((535, 263), (500, 359), "#662D91")
wf.add_text((671, 473, 158, 69), "Get some measures\non the classification experiment.", 16)
wf.add_arrow((730, 472), (674, 420), "#39B54A")
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
