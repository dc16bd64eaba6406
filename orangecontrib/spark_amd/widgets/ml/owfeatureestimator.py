"""Feature Estimator widget: reflective Estimator over
orange3_spark_amd.ml.feature (reference widgets/ml/spark_ml_feature.py where it exists)."""
from orange3_spark_amd.ml import feature

from ..base import OWEstimatorBase


class OWFeatureEstimator(OWEstimatorBase):
    priority = 7
    name = "Feature Estimator"
    description = "Fit any estimator of ml.feature"
    icon = "../icons/feature.svg"
    module = feature
    box_text = "Feature Estimator"


from ..views import export_views  # noqa: E402

export_views(globals())
