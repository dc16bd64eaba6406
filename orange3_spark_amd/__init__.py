"""orange3_spark_amd -- an MI355X-native visual-workflow ML backend.

Same capabilities as Orange3-Spark (reference: Gjerman/Orange3-Spark), re-designed for
AMD Instinct MI355X (gfx950): a row-sharded columnar DataFrame engine in HBM,
hand-written CDNA4 HIP kernels for the hot estimators, RCCL (torch.distributed
"nccl") collectives over xGMI, and a pyspark.ml-compatible Param/Estimator/Transformer/
Pipeline API with Spark-format model persistence.

Quick start::

    from orange3_spark_amd import Session
    from orange3_spark_amd.ml.classification import LogisticRegression
    s = Session.getOrCreate()
    df = s.synthetic.classification(1_000_000, 256)
    model = LogisticRegression(maxIter=20).fit(df)
"""
from .conf import SessionConf, SparkConf  # noqa: F401
from .session import Session, SparkSession, __version__  # noqa: F401
from .frame.dataframe import DataFrame, Row  # noqa: F401
from .frame import expr as functions  # noqa: F401
