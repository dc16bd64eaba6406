"""Classification widget: reflective Estimator over
orange3_spark_amd.ml.classification (reference widgets/ml/spark_ml_classification.py where it exists)."""
from orange3_spark_amd.ml import classification

from ..base import OWEstimatorBase


class OWClassification(OWEstimatorBase):
    priority = 1
    name = "Classification"
    description = "Fit any estimator of ml.classification"
    icon = "../icons/classify.svg"
    module = classification
    box_text = "Classification"


from ..views import export_views  # noqa: E402

export_views(globals())
