"""``pyspark.ml.pipeline`` import path: Pipeline / PipelineModel live in :mod:`.base` (the
reference reaches them through ``pyspark.ml``; scripts written against Spark also import
``from pyspark.ml.pipeline import Pipeline, PipelineModel``)."""
from .base import Estimator, Model, Pipeline, PipelineModel, Transformer  # noqa: F401

__all__ = ["Pipeline", "PipelineModel", "Estimator", "Model", "Transformer"]
