"""``pyspark.ml.torch`` counterpart: :class:`TorchDistributor`."""
from .distributor import TorchDistributor

__all__ = ["TorchDistributor"]
