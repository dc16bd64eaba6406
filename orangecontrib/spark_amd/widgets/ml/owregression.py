"""Regression widget: reflective Estimator over
orange3_spark_amd.ml.regression (reference widgets/ml/spark_ml_regression.py where it exists)."""
from orange3_spark_amd.ml import regression

from ..base import OWEstimatorBase


class OWRegression(OWEstimatorBase):
    priority = 3
    name = "Regression"
    description = "Fit any estimator of ml.regression"
    icon = "../icons/regression.svg"
    module = regression
    box_text = "Regression"


from ..views import export_views  # noqa: E402

export_views(globals())
