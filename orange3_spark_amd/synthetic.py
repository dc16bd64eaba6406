"""Synthetic datasets for the BASELINE configs, generated on device from counter hashes.

Rows are a pure function of (seed, global row index), so a dataset is identical for any
number of GPUs and any partitioning.  Large datasets can exceed one GPU's HBM (1B x 256
bf16 = 512 GB vs 288 GB): such a DataFrame keeps as many rows *resident* in HBM as the
cache budget allows and marks the rest as *lineage* rows that consumers recompute
in-kernel on every pass.  This is Spark's ``MEMORY_ONLY`` storage-level semantics
(partitions that do not fit are recomputed from lineage when used), done at HBM scale.
"""
from __future__ import annotations

from collections import OrderedDict
from dataclasses import dataclass

import numpy as np
import torch

from .frame import column as C
from .frame.dataframe import DataFrame
from .ops import glm as G


@dataclass
class GlmSpec:
    seed: int
    d: int          # logical feature count (rounded up to a multiple of 8)
    ld: int
    wtrue: torch.Tensor
    btrue: float


class LineageVectorColumn(C.VectorColumn):
    """Vector column whose rows [resident, n) are regenerated from ``spec`` on demand.

    ``data`` holds the resident prefix only; ``row0`` is the global index of local row 0.
    Operations that need arbitrary rows materialise them (bounded by ``max_materialise``).
    """

    max_materialise_bytes = 32 << 30

    def __init__(self, spec: GlmSpec, n: int, row0: int, resident: torch.Tensor):
        super().__init__(resident, spec.ld)
        self.spec, self._n, self.row0 = spec, int(n), int(row0)

    def __len__(self):
        return self._n

    @property
    def resident_rows(self) -> int:
        return int(self.data.shape[0])

    @property
    def lineage_rows(self) -> int:
        return self._n - self.resident_rows

    def _gen(self, start: int, end: int) -> torch.Tensor:
        X, _ = G.synth_glm(end - start, self.spec.d, self.spec.seed, self.row0 + start, self.data.device,
                           self.spec.ld, self.spec.wtrue, self.spec.btrue)
        return X

    def full(self) -> torch.Tensor:
        if self.lineage_rows == 0:
            return self.data
        nbytes = self._n * self.ld * 2
        if nbytes > self.max_materialise_bytes:
            raise MemoryError(f"materialising {nbytes / 2**30:.1f} GiB of lineage rows; consume this column "
                              f"with a lineage-aware op (GLM solvers) or sample/limit first")
        return torch.cat([self.data, self._gen(self.resident_rows, self._n)])

    def dense(self):
        return self.full()

    def take(self, idx):
        if self.lineage_rows == 0:
            return C.VectorColumn(self.data[idx.to(self.data.device)], self.size)
        idx = idx.to(torch.int64)
        fk = G.feat_keys(self.spec.seed, idx.to(self.data.device) + self.row0)
        return C.VectorColumn(G.synth_features_torch(fk, self.ld, self.spec.d), self.size)

    def mask_select(self, mask):
        return self.take(torch.nonzero(mask.to(self.data.device)).reshape(-1))

    def slice(self, start, end):
        start, end = max(0, start), min(self._n, end)
        if end <= self.resident_rows:
            return C.VectorColumn(self.data[start:end], self.size)
        res = self.data[start:min(end, self.resident_rows)]
        return LineageVectorColumn(self.spec, end - start, self.row0 + start, res)

    def to_numpy(self):
        return C.VectorColumn(self.full(), self.size).to_numpy()

    def materialise(self, budget_bytes: int) -> None:
        """Grow the resident prefix up to ``budget_bytes`` of HBM."""
        want = min(self._n, max(self.resident_rows, int(budget_bytes // (self.ld * 2))))
        if want > self.resident_rows:
            extra = self._gen(self.resident_rows, want)
            self.data = torch.cat([self.data, extra]) if self.resident_rows else extra

    @staticmethod
    def concat(cols):
        return C.VectorColumn(torch.cat([c.full() if isinstance(c, LineageVectorColumn) else c.data for c in cols]),
                              cols[0].size)


class GlmLineage:
    """Attached to a synthetic DataFrame: resolves resident rows on ``cache()``."""

    def __init__(self, col_name: str, budget_fraction: float):
        self.col_name = col_name
        self.fraction = budget_fraction

    def materialise(self, df: DataFrame) -> None:
        c = df._cols.get(self.col_name)
        if not isinstance(c, LineageVectorColumn):
            return
        dev = c.data.device
        if dev.type == "cuda":
            free, _ = torch.cuda.mem_get_info(dev)
            budget = int(free * self.fraction) + c.resident_rows * c.ld * 2
        else:
            budget = 8 << 30
        c.materialise(budget)


class SyntheticData:
    """``session.synthetic.*`` generators (each rank generates only its own rows)."""

    def __init__(self, session):
        self.session = session

    def _bounds(self, n: int) -> tuple[int, int]:
        return self.session._shard_bounds(n)

    def classification(self, numRows: int, numFeatures: int, seed: int = 42, cache: bool = True,
                       resident_fraction: float | None = None) -> DataFrame:
        """Binary classification rows: features U[-1,1) (bf16 on GPU), label ~ Bernoulli(
        sigmoid(x.w* + b*)).  Columns: ``features`` (vector), ``label`` (float)."""
        s = self.session
        d = G.padded_width(numFeatures)
        wt, bt = G.synth_truth(seed, numFeatures, d)
        spec = GlmSpec(seed, d, d, wt, bt)
        lo, hi = self._bounds(numRows)
        n = hi - lo
        dev = s.device
        frac = s.conf.memory_fraction() if resident_fraction is None else resident_fraction
        # labels are always materialised (4 B/row); features up to the HBM budget
        y = torch.empty(n, dtype=torch.float32, device=dev)
        if dev.type == "cuda":
            free, _ = torch.cuda.mem_get_info(dev)
            budget = max(0, int(free * frac) - n * 4)
            resident = min(n, budget // (d * 2)) if cache else 0
        else:
            resident = n
        X = torch.empty((resident, d), dtype=torch.bfloat16, device=dev)
        step = 1 << 26 if dev.type == "cuda" else 1 << 16
        for a in range(0, n, step):
            b = min(n, a + step)
            if dev.type == "cuda" and a >= resident:
                # labels only (features stay lineage): generate into a scratch chunk
                Xc, yc = G.synth_glm(b - a, d, seed, lo + a, dev, d, wt, bt)
                y[a:b] = yc
                del Xc
                continue
            e = min(b, resident)
            Xc, yc = G.synth_glm(b - a, d, seed, lo + a, dev, d, wt, bt)
            X[a:e] = Xc[: e - a]
            y[a:b] = yc
            del Xc
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        feat = LineageVectorColumn(spec, n, lo, X) if resident < n else C.VectorColumn(X, d)
        if dev.type != "cuda":
            feat = C.VectorColumn(X.to(s.vector_dtype()), d)
        df = DataFrame(s, OrderedDict(features=feat, label=C.NumericColumn(y)), n)
        df.lineage = GlmLineage("features", frac)
        df.synthetic_spec = spec
        return df

    def table(self, numRows: int, numFeatures: int, seed: int = 42, dtype=torch.float32,
              prefix: str = "f") -> DataFrame:
        """A wide columnar table (what a parquet / Hive table read gives): one numeric column
        per feature (``f0..f{d-1}``, ``dtype``) and a float ``label`` -- the same rows as
        :meth:`classification` (so the assembled features equal its feature vectors), but
        stored column by column, for the DatasetBuilder -> VectorAssembler path."""
        s = self.session
        d = G.padded_width(numFeatures)
        wt, bt = G.synth_truth(seed, numFeatures, d)
        lo, hi = self._bounds(numRows)
        n = hi - lo
        dev = s.device
        cols = [torch.empty(n, dtype=dtype, device=dev) for _ in range(numFeatures)]
        y = torch.empty(n, dtype=torch.float32, device=dev)
        step = 1 << 23 if dev.type == "cuda" else 1 << 16
        for a in range(0, n, step):
            b = min(n, a + step)
            Xc, yc = G.synth_glm(b - a, d, seed, lo + a, dev, d, wt, bt)
            for j in range(numFeatures):
                cols[j][a:b] = Xc[:, j]
            y[a:b] = yc
            del Xc
        out = OrderedDict((f"{prefix}{j}", C.NumericColumn(cols[j])) for j in range(numFeatures))
        out["label"] = C.NumericColumn(y)
        return DataFrame(s, out, n)

    def blobs(self, numRows: int, numFeatures: int, k: int, seed: int = 42, spread: float = 1.0,
              dtype=torch.float32) -> DataFrame:
        """Gaussian blobs around k centres (KMeans config): ``features`` f32 [n, d]."""
        s = self.session
        lo, hi = self._bounds(numRows)
        dev = s.device
        gen = torch.Generator(device="cpu").manual_seed(seed)
        centers = (torch.rand((k, numFeatures), generator=gen, dtype=torch.float64) * 20 - 10).to(dev, dtype)
        n = hi - lo
        X = torch.empty((n, numFeatures), dtype=dtype, device=dev)
        lab = torch.empty(n, dtype=torch.int32, device=dev)
        step = 1 << 20
        cols = torch.arange(numFeatures, dtype=torch.int64, device=dev)
        for a in range(0, n, step):
            b = min(n, a + step)
            rows = torch.arange(lo + a, lo + b, dtype=torch.int64, device=dev)
            cid = (G.row_keys(seed, rows) % k).to(torch.int64)
            # Box-Muller noise keyed on (row, column): identical for any partitioning
            key = rows[:, None] * numFeatures + cols[None, :]
            h1 = G.row_keys(seed ^ 0x3C6EF372, key.reshape(-1))
            h2 = G._fmix32(h1 ^ 0x1B873593)
            u1 = ((h1 >> 8).to(torch.float32) + 0.5) * (1.0 / 16777216.0)
            u2 = (h2 >> 8).to(torch.float32) * (1.0 / 16777216.0)
            z = torch.sqrt(-2.0 * torch.log(u1)) * torch.cos(6.283185307179586 * u2)
            X[a:b] = centers[cid] + spread * z.reshape(b - a, numFeatures).to(dtype)
            lab[a:b] = cid.to(torch.int32)
        df = DataFrame(s, OrderedDict(features=C.VectorColumn(X), cluster=C.NumericColumn(lab)), n)
        df.true_centers = centers
        return df

    def ratings(self, numUsers: int, numItems: int, numRatings: int, rank: int = 8, seed: int = 42,
                implicit: bool = False) -> DataFrame:
        """(user, item, rating) triples from a low-rank model (ALS config)."""
        s = self.session
        lo, hi = self._bounds(numRatings)
        dev = s.device
        n = hi - lo
        rows = torch.arange(lo, hi, dtype=torch.int64, device=dev)
        ku = G.row_keys(seed, rows)
        ki = G.row_keys(seed ^ 0x1234567, rows)
        users = (ku % numUsers).to(torch.int32)
        items = (ki % numItems).to(torch.int32)
        gen = torch.Generator(device="cpu").manual_seed(seed)
        U = (torch.randn((numUsers, rank), generator=gen) / np.sqrt(rank)).to(dev) if numUsers * rank <= 1 << 28 else None
        V = (torch.randn((numItems, rank), generator=gen) / np.sqrt(rank)).to(dev) if numItems * rank <= 1 << 28 else None
        if U is not None and V is not None:
            r = (U[users.long()] * V[items.long()]).sum(1) * 2 + 3
        else:
            r = (G.row_keys(seed ^ 0x55, rows) % 5 + 1).to(torch.float32)
        if implicit:
            r = torch.clamp(r, min=0.0)
        df = DataFrame(s, OrderedDict(user=C.NumericColumn(users), item=C.NumericColumn(items),
                                      rating=C.NumericColumn(r.to(torch.float32))), n)
        return df

    def trees(self, numRows: int, numFeatures: int, seed: int = 42) -> DataFrame:
        """Nonlinear binary classification (GBT/RF config): ``features`` (the session's vector
        storage dtype: bf16 on the GPU -- the 256-level synthetic values are exact in bf16,
        so 500M x 64 holds 64 GB instead of 128), ``label``."""
        s = self.session
        lo, hi = self._bounds(numRows)
        dev = s.device
        n = hi - lo
        vdt = s.vector_dtype()
        X = torch.empty((n, numFeatures), dtype=vdt if vdt in (torch.bfloat16, torch.float32) else torch.float32,
                        device=dev)
        y = torch.empty(n, dtype=torch.float32, device=dev)
        step = 1 << 24
        for a in range(0, n, step):
            b = min(n, a + step)
            rk = G.row_keys(seed, torch.arange(lo + a, lo + b, dtype=torch.int64, device=dev))
            xb = G.synth_features_torch(rk, G.padded_width(numFeatures), numFeatures)[:, :numFeatures].float()
            X[a:b] = xb.to(X.dtype)
            score = torch.sin(3 * xb[:, 0]) + xb[:, 1] * xb[:, 2] * 2 - (xb[:, 3 % numFeatures] > 0.3).float()
            u = ((G._fmix32(rk ^ 0x7777) >> 8).float() / 16777216.0)
            y[a:b] = (u < torch.sigmoid(2 * score)).float()
        return DataFrame(s, OrderedDict(features=C.VectorColumn(X), label=C.NumericColumn(y)), n)
