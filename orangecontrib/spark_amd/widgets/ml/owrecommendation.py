"""Recommendation widget: reflective Estimator over
orange3_spark_amd.ml.recommendation (reference widgets/ml/spark_ml_recommendation.py where it exists)."""
from orange3_spark_amd.ml import recommendation

from ..base import OWEstimatorBase


class OWRecommendation(OWEstimatorBase):
    priority = 4
    name = "Recommendation"
    description = "Fit any estimator of ml.recommendation"
    icon = "../icons/recommend.svg"
    module = recommendation
    box_text = "Recommendation"


from ..views import export_views  # noqa: E402

export_views(globals())
