"""Frequent Patterns widget: reflective Estimator over
orange3_spark_amd.ml.fpm (reference widgets/ml/spark_ml_fpm.py where it exists)."""
from orange3_spark_amd.ml import fpm

from ..base import OWEstimatorBase


class OWFrequentPatterns(OWEstimatorBase):
    priority = 12
    name = "Frequent Patterns"
    description = "Fit any estimator of ml.fpm"
    icon = "../icons/feature.svg"
    module = fpm
    box_text = "Frequent Patterns"


from ..views import export_views  # noqa: E402

export_views(globals())
