"""Feature widget: reflective Transformer over
orange3_spark_amd.ml.feature (reference widgets/ml/spark_ml_feature.py where it exists)."""
from orange3_spark_amd.ml import feature

from ..base import OWTransformerBase


class OWFeature(OWTransformerBase):
    priority = 6
    name = "Feature"
    description = "Apply any transformer of ml.feature"
    icon = "../icons/feature.svg"
    module = feature
    box_text = "Feature"


from ..views import export_views  # noqa: E402

export_views(globals())
