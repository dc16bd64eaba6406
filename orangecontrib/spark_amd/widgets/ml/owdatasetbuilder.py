"""Dataset Builder: assign columns to features / label / metas, then VectorAssembler
(reference widgets/ml/spark_ml_dataset.py:292-593; ``commit`` :569-582).  Quirk fixes
(Q5): the column lists are cleared on new input, metas are passed through (kept as
columns), and role hints are restored when the same columns arrive again."""
from orange3_spark_amd.frame.dataframe import DataFrame
from orange3_spark_amd.ml.feature import VectorAssembler

from ..compat import Setting, Widget


class OWDatasetBuilder(Widget):
    priority = 5
    name = "Dataset Builder"
    description = "Assemble a features vector and a label column"
    icon = "../icons/builder.svg"
    inputs = [("DataFrame", DataFrame, "set_data")]
    outputs = [("DataFrame", DataFrame)]
    domain_role_hints = Setting({})
    featuresCol = Setting("features")
    labelCol = Setting("label")

    def __init__(self, **kw):
        super().__init__(**kw)
        self.in_df = None
        self.available_attrs, self.used_attrs, self.class_attrs, self.meta_attrs = [], [], [], []

    def set_data(self, df):
        self.in_df = df
        self.available_attrs, self.used_attrs, self.class_attrs, self.meta_attrs = [], [], [], []
        if df is None:
            return
        hints = self.domain_role_hints.get(tuple(df.columns))
        if hints:
            self.used_attrs = list(hints["features"])
            self.class_attrs = list(hints["label"])
            self.meta_attrs = list(hints["metas"])
        used = set(self.used_attrs) | set(self.class_attrs) | set(self.meta_attrs)
        self.available_attrs = [c for c in df.columns if c not in used]

    def _move(self, names, dst):
        for n in names:
            for lst in (self.available_attrs, self.used_attrs, self.class_attrs, self.meta_attrs):
                if n in lst:
                    lst.remove(n)
            dst.append(n)

    def set_features(self, names):
        self._move(names, self.used_attrs)

    def set_label(self, name):
        self._move(self.class_attrs[:], self.available_attrs)   # at most one label
        if name is not None:
            self._move([name], self.class_attrs)

    def set_metas(self, names):
        self._move(names, self.meta_attrs)

    def move_to_available(self, names):
        """Return columns from any role list to the available list (canvas "< Available")."""
        self._move(names, self.available_attrs)

    def move_feature(self, name, delta: int):
        """Reorder the features list (canvas Up / Down): the assembled vector follows it."""
        if name in self.used_attrs:
            i = self.used_attrs.index(name)
            j = max(0, min(len(self.used_attrs) - 1, i + int(delta)))
            self.used_attrs.insert(j, self.used_attrs.pop(i))

    def filtered_available(self, pattern: str = "") -> list:
        """Available columns whose name contains every whitespace-separated word of
        ``pattern`` (case-insensitive) -- the reference's filter line edit (:537-567)."""
        words = [w.lower() for w in (pattern or "").split()]
        return [c for c in self.available_attrs if all(w in c.lower() for w in words)]

    def update_domain_role_hints(self):
        if self.in_df is not None:
            self.domain_role_hints[tuple(self.in_df.columns)] = {
                "features": list(self.used_attrs), "label": list(self.class_attrs), "metas": list(self.meta_attrs)}

    def commit(self):
        self.update_domain_role_hints()
        if self.in_df is None:
            self.send("DataFrame", None)
            return None
        out = VectorAssembler(inputCols=list(self.used_attrs), outputCol=self.featuresCol).transform(self.in_df)
        if self.class_attrs:
            out = out.withColumn(self.labelCol, out[self.class_attrs[0]].cast("double"))
        keep = [self.featuresCol] + ([self.labelCol] if self.class_attrs else []) + \
            [m for m in self.meta_attrs if m not in (self.featuresCol, self.labelCol)]
        rest = [c for c in out.columns if c not in keep]
        out = out.select(*(rest + keep))
        self.send("DataFrame", out)
        return out

    def reset(self):
        if self.in_df is not None:
            self.available_attrs = list(self.in_df.columns)
        else:
            self.available_attrs = []
        self.used_attrs, self.class_attrs, self.meta_attrs = [], [], []
        self.update_domain_role_hints()


from ..views import export_views  # noqa: E402

export_views(globals())
