"""Model Save/Load widget (beyond-ref): Spark-format ``save``/``load`` of any model or
pipeline (metadata JSON + parquet data)."""
from orange3_spark_amd.ml.base import Model
from orange3_spark_amd.ml.util import MLReader, load_metadata, py_class

from ..compat import Setting, Widget


class OWModelIO(Widget):
    priority = 11
    name = "Model Save/Load"
    description = "Save a model in Spark ML format, or load one"
    icon = "../icons/save.svg"
    inputs = [("Model", Model, "set_model")]
    outputs = [("Model", Model)]
    path = Setting("")
    overwrite = Setting(True)

    def __init__(self, **kw):
        super().__init__(**kw)
        self.model = None

    def set_model(self, model):
        self.model = model

    def save(self, path=None):
        path = path or self.path
        w = self.model.write()
        if self.overwrite:
            w = w.overwrite()
        w.save(path)
        self.path = path
        return path

    def load(self, path=None):
        path = path or self.path
        cls = py_class(load_metadata(path)["class"])
        self.model = MLReader(cls).load(path)
        self.path = path
        self.send("Model", self.model)
        return self.model


from ..views import export_views  # noqa: E402

export_views(globals())
