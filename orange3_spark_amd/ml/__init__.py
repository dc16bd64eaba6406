"""pyspark.ml-compatible ML API (Estimator/Transformer/Model/Evaluator/Pipeline)."""
from .base import Estimator, Evaluator, Model, Pipeline, PipelineModel, Transformer, UnaryTransformer  # noqa: F401
