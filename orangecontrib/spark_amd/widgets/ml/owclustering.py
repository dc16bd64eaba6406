"""Clustering widget: reflective Estimator over
orange3_spark_amd.ml.clustering (reference widgets/ml/spark_ml_clustering.py where it exists)."""
from orange3_spark_amd.ml import clustering

from ..base import OWEstimatorBase


class OWClustering(OWEstimatorBase):
    priority = 2
    name = "Clustering"
    description = "Fit any estimator of ml.clustering"
    icon = "../icons/kmeans.svg"
    module = clustering
    box_text = "Clustering"


from ..views import export_views  # noqa: E402

export_views(globals())
