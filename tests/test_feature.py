"""Feature transformers/estimators on the CPU path vs numpy / scikit-learn / Spark-doc values."""
import numpy as np
import pandas as pd
import pytest
import torch

from orange3_spark_amd import Session, SessionConf
from orange3_spark_amd.ml import feature as F
from orange3_spark_amd.ml.base import Pipeline, PipelineModel
from orange3_spark_amd.ml.classification import LogisticRegression


@pytest.fixture(scope="module")
def s():
    return Session(SessionConf().set("o3s.device", "cpu"))


def test_hashing_tf_matches_spark_doc_example(s):
    df = s.createDataFrame(pd.DataFrame({"words": [["a", "b", "c"]]}))
    out = F.HashingTF(numFeatures=10, inputCol="words", outputCol="features").transform(df)
    v = out.collect()[0].features
    assert list(v.indices) == [5, 7, 8] and list(v.values) == [1.0, 1.0, 1.0]


def test_tokenizer_stopwords_ngram_countvectorizer_idf(s):
    df = s.createDataFrame(pd.DataFrame({"text": ["Hello world of Spark", "the quick brown fox", "hello hello"]}))
    tok = F.Tokenizer(inputCol="text", outputCol="words").transform(df)
    assert tok.collect()[0].words == ["hello", "world", "of", "spark"]
    sw = F.StopWordsRemover(inputCol="words", outputCol="clean").transform(tok)
    assert sw.collect()[1].clean == ["quick", "brown", "fox"]
    ng = F.NGram(n=2, inputCol="words", outputCol="ng").transform(tok)
    assert ng.collect()[2].ng == ["hello hello"]
    cvm = F.CountVectorizer(inputCol="words", outputCol="tf").fit(tok)
    assert cvm.vocabulary[0] == "hello"
    tf = cvm.transform(tok)
    idf = F.IDF(inputCol="tf", outputCol="tfidf").fit(tf)
    out = idf.transform(tf).collect()
    assert np.isclose(idf.idf.toArray()[0], np.log(4 / 3))
    assert out[2].tfidf.values[0] == pytest.approx(2 * np.log(4 / 3))
    rt = F.RegexTokenizer(inputCol="text", outputCol="w2", pattern="\\W+").transform(df)
    assert rt.collect()[0].w2 == ["hello", "world", "of", "spark"]


def test_scalers_match_sklearn(s):
    from sklearn.preprocessing import MaxAbsScaler, MinMaxScaler, StandardScaler
    rng = np.random.default_rng(0)
    X = rng.normal(size=(200, 4)) * [1, 2, 3, 4] + [0, 1, 2, 3]
    df = s.createDataFrame(pd.DataFrame({"f": list(X)}))
    ss = F.StandardScaler(inputCol="f", outputCol="o", withMean=True).fit(df).transform(df)
    got = np.stack([r.o.toArray() for r in ss.collect()])
    ref = (X - X.mean(0)) / X.std(0, ddof=1)
    assert np.allclose(got, ref)
    mm = F.MinMaxScaler(inputCol="f", outputCol="o").fit(df).transform(df)
    assert np.allclose(np.stack([r.o.toArray() for r in mm.collect()]), MinMaxScaler().fit_transform(X))
    ma = F.MaxAbsScaler(inputCol="f", outputCol="o").fit(df).transform(df)
    assert np.allclose(np.stack([r.o.toArray() for r in ma.collect()]), MaxAbsScaler().fit_transform(X))


def test_string_indexer_onehot_index_to_string(s):
    df = s.createDataFrame(pd.DataFrame({"c": ["a", "b", "a", "c", "a", "c"]}))
    m = F.StringIndexer(inputCol="c", outputCol="ci").fit(df)
    assert m.labels == ["a", "c", "b"]
    out = m.transform(df)
    assert [r.ci for r in out.collect()] == [0.0, 2.0, 0.0, 1.0, 0.0, 1.0]
    oh = F.OneHotEncoder(inputCols=["ci"], outputCols=["oh"]).fit(out).transform(out)
    v = oh.collect()[1].oh
    assert v.size == 2 and v.toArray().tolist() == [0.0, 0.0]
    back = F.IndexToString(inputCol="ci", outputCol="orig", labels=m.labels).transform(out)
    assert [r.orig for r in back.collect()] == ["a", "b", "a", "c", "a", "c"]


def test_pca_matches_numpy(s):
    rng = np.random.default_rng(1)
    X = rng.normal(size=(300, 5)) @ rng.normal(size=(5, 5))
    df = s.createDataFrame(pd.DataFrame({"f": list(X)}))
    m = F.PCA(k=2, inputCol="f", outputCol="p").fit(df)
    w, v = np.linalg.eigh(np.cov(X.T))
    top = v[:, np.argsort(w)[::-1][:2]]
    assert np.allclose(np.abs(m.pc.toArray()), np.abs(top), atol=1e-8)


def test_misc_transformers(s):
    df = s.createDataFrame(pd.DataFrame({"x": [0.1, 0.6, 1.5], "v": [np.array([1.0, 2.0])] * 3}))
    assert [r.b for r in F.Binarizer(threshold=0.5, inputCol="x", outputCol="b").transform(df).collect()] == [0, 1, 1]
    bz = F.Bucketizer(splits=[-np.inf, 0.5, 1.0, np.inf], inputCol="x", outputCol="b").transform(df)
    assert [r.b for r in bz.collect()] == [0.0, 1.0, 2.0]
    pe = F.PolynomialExpansion(degree=2, inputCol="v", outputCol="p").transform(df).collect()[0].p.toArray()
    assert pe.tolist() == [1.0, 1.0, 2.0, 2.0, 4.0]     # Spark order: x, x^2, y, xy, y^2
    nz = F.Normalizer(p=1.0, inputCol="v", outputCol="n").transform(df).collect()[0].n.toArray()
    assert np.allclose(nz, [1 / 3, 2 / 3])
    ew = F.ElementwiseProduct(scalingVec=[2.0, 3.0], inputCol="v", outputCol="e").transform(df)
    assert ew.collect()[0].e.toArray().tolist() == [2.0, 6.0]
    dct = F.DCT(inputCol="v", outputCol="d").transform(df).collect()[0].d.toArray()
    from scipy.fft import dct as sdct
    assert np.allclose(dct, sdct(np.array([1.0, 2.0]), norm="ortho"))
    imp = F.Imputer(inputCols=["x"], outputCols=["xi"], strategy="median").fit(df)
    assert imp.surrogates["x"] == 0.6


def test_pipeline_fit_save_load(s, tmp_path):
    rng = np.random.default_rng(2)
    X = rng.normal(size=(400, 3))
    y = (X @ [1, -2, 0.5] > 0).astype(float)
    df = s.createDataFrame(pd.DataFrame({"a": X[:, 0], "b": X[:, 1], "c": X[:, 2], "label": y}))
    pipe = Pipeline(stages=[F.VectorAssembler(inputCols=["a", "b", "c"], outputCol="raw"),
                            F.StandardScaler(inputCol="raw", outputCol="features"),
                            LogisticRegression(maxIter=50)])
    pm = pipe.fit(df)
    acc = (pm.transform(df).toPandas()["prediction"].values == y).mean()
    assert acc > 0.95
    pm.save(str(tmp_path / "pm"))
    pm2 = PipelineModel.load(str(tmp_path / "pm"))
    p1 = pm.transform(df).toPandas()["prediction"].values
    p2 = pm2.transform(df).toPandas()["prediction"].values
    assert np.array_equal(p1, p2)
    import json
    meta = json.loads(open(tmp_path / "pm" / "metadata" / "part-00000").read())
    assert meta["class"] == "org.apache.spark.ml.PipelineModel" and len(meta["paramMap"]["stageUids"]) == 3
    pipe.save(str(tmp_path / "p"))
    p3 = Pipeline.load(str(tmp_path / "p"))
    assert [type(x).__name__ for x in p3.getStages()] == ["VectorAssembler", "StandardScaler", "LogisticRegression"]


def test_tokenizer_spark_split_semantics(s):
    """Spark Tokenizer = toLowerCase + split("\\\\s"): whitespace runs give empty tokens,
    trailing empties dropped, "" -> [""], all-whitespace -> []."""
    from orange3_spark_amd.ops.text import spark_split, tokenize_lower_ws
    cases = ["a  b", " a", "a ", "   ", "", "Tab\tSep\nLine", "x\x0by\x0cz\rw", "MiXeD  Case  "]
    want = [["a", "", "b"], ["", "a"], ["a"], [], [""], ["tab", "sep", "line"], ["x", "y", "z", "w"],
            ["mixed", "", "case"]]
    assert [spark_split(c.lower()) for c in cases] == want
    assert tokenize_lower_ws(cases + [None]) == want + [None]
    assert tokenize_lower_ws(["Ünïcode  Straße"]) == [["ünïcode", "", "straße"]]


def _corpus(n, seed):
    rng = np.random.default_rng(seed)
    words = ["Spark", "GPU", "mi355x", "HashingTF", "the", "a", "", "x" * 40, "Tok3n", "UPPER"]
    seps = [" ", "  ", "\t", "\n", " \r ", "\x0b"]
    out = []
    for i in range(n):
        k = int(rng.integers(0, 12))
        parts = [words[int(j)] for j in rng.integers(0, len(words), k)]
        txt = ""
        for p in parts:
            txt += p + seps[int(rng.integers(0, len(seps)))]
        if rng.uniform() < 0.2:
            txt = seps[int(rng.integers(0, len(seps)))] + txt
        if rng.uniform() < 0.3:
            txt = txt.rstrip()
        out.append(None if i % 97 == 5 else txt)
    return out


@pytest.mark.gpu
def test_gpu_tokenizer_and_hashingtf_match_host():
    """Device Tokenizer (tokenize kernels) + HashingTF over the device token spans ==
    the host path, token for token and CSR entry for entry."""
    from orange3_spark_amd import Session, SessionConf
    from orange3_spark_amd.frame import column as C
    from orange3_spark_amd.ops.text import tokenize_lower_ws
    gs = Session(SessionConf().set("o3s.device", "cuda"))
    texts = _corpus(20_011, 3)
    df = gs.createDataFrame(pd.DataFrame({"text": texts}))
    tok = F.Tokenizer(inputCol="text", outputCol="words").transform(df)
    col = tok.column_data("words")
    assert isinstance(col, C.DeviceTokensColumn)
    assert list(col.values) == tokenize_lower_ws(texts)
    tf = F.HashingTF(numFeatures=1 << 12, inputCol="words", outputCol="tf").transform(tok).column_data("tf")
    host = F._terms_to_csr([None if v is None else v for v in tokenize_lower_ws(texts)], 1 << 12,
                           torch.device("cpu"), False)
    assert torch.equal(tf.indptr.cpu(), host.indptr.cpu())
    assert torch.equal(tf.indices.cpu(), host.indices.cpu())
    assert torch.equal(tf.values.cpu(), host.values.cpu())
    # downstream host consumers still work on the lazily decoded lists
    sw = F.StopWordsRemover(inputCol="words", outputCol="clean").transform(tok)
    assert sw.count() == len(texts)


@pytest.mark.gpu
@pytest.mark.parametrize("binary", [False, True])
def test_gpu_hashingtf_per_document_kernel_edges(binary):
    """hashing_tf_*_kernel (one wave per document: register bitonic sort <= 64 tokens, LDS
    sort <= 4096, torch above) == the global (row, bucket) sort, bitwise: documents of 0,
    1, 63, 64, 65, 127, 4096, 4097 and 6000 tokens, heavy duplicates (small vocabularies)
    and a tiny numFeatures (many collisions)."""
    from orange3_spark_amd import Session, SessionConf
    from orange3_spark_amd.frame import column as C
    from orange3_spark_amd.ops import text as TX
    gs = Session(SessionConf().set("o3s.device", "cuda"))
    rng = np.random.default_rng(7)
    lens = [0, 1, 63, 64, 65, 127, 4096, 4097, 6000] + list(rng.integers(0, 300, 400))
    texts = []
    for i, L in enumerate(lens):
        vocab = 5 if i % 3 == 0 else 2000
        texts.append(" ".join(f"t{int(v)}" for v in rng.integers(0, vocab, L)) if L else "")
    df = gs.createDataFrame(pd.DataFrame({"text": texts}))
    col = F.Tokenizer(inputCol="text", outputCol="w").transform(df).column_data("w")
    assert isinstance(col, C.DeviceTokensColumn)
    for nf in (1 << 18, 37):
        indptr, idx, val = TX.hashing_tf_csr(col, nf, binary)
        bucket = TX.murmur3_span_buckets(col, nf)
        ref = F._buckets_to_csr(bucket, col.doc_offs[1:] - col.doc_offs[:-1], len(col), nf, binary)
        assert torch.equal(indptr, ref.indptr) and torch.equal(idx, ref.indices) and torch.equal(val, ref.values)


@pytest.mark.gpu
@pytest.mark.parametrize("handle", ["keep", "skip", "error"])
def test_gpu_vector_assembler_fused_kernel_matches_torch(handle):
    """The one-pass assemble kernel (any dtype, null masks, vector inputs, padded bf16 out)
    == the torch composition on the same columns, for every handleInvalid mode."""
    import numpy as np
    import torch
    from collections import OrderedDict
    from orange3_spark_amd import Session, SessionConf
    from orange3_spark_amd.frame import column as C
    from orange3_spark_amd.frame.dataframe import DataFrame
    from orange3_spark_amd.ml.feature import VectorAssembler
    dev = torch.device("cuda", 0)
    s = Session(SessionConf().setAppName("asm"), device=dev)
    g = torch.Generator().manual_seed(1)
    n = 100_003
    f64 = torch.randn(n, generator=g, dtype=torch.float64)
    f32 = torch.randn(n, generator=g)
    i64 = torch.randint(-5, 5, (n,), generator=g)
    i32 = torch.randint(0, 100, (n,), generator=g, dtype=torch.int32)
    bo = torch.rand(n, generator=g) > 0.5
    vec = torch.randn((n, 12), generator=g).to(torch.bfloat16)
    vec_pad = torch.zeros((n, 16), dtype=torch.bfloat16)
    vec_pad[:, :12] = vec
    valid = torch.ones(n, dtype=torch.bool)
    if handle != "keep" or True:
        valid[::997] = False
    f64[5] = float("nan")
    cols = OrderedDict(a=C.NumericColumn(f64.to(dev)), b=C.NumericColumn(f32.to(dev), valid.to(dev)),
                       c=C.NumericColumn(i64.to(dev)), d=C.NumericColumn(i32.to(dev)), e=C.NumericColumn(bo.to(dev)),
                       v=C.VectorColumn(vec_pad.to(dev), 12), lab=C.NumericColumn(torch.arange(n, dtype=torch.float64).to(dev)))
    df = DataFrame(s, cols, n)
    va = VectorAssembler(inputCols=["a", "b", "c", "d", "e", "v"], outputCol="f", handleInvalid=handle)
    ref_rows = torch.stack([f64, torch.where(valid, f32.double(), torch.full_like(f64, float("nan"))), i64.double(),
                            i32.double(), bo.double()], 1)
    ref = torch.cat([ref_rows, vec.double()], 1)
    bad = torch.isnan(ref).any(1)
    if handle == "error":
        with pytest.raises(ValueError, match="handleInvalid"):
            va.transform(df)
        return
    out = va.transform(df)
    col = out.column_data("f")
    assert col.size == 17 and col.data.dtype == torch.bfloat16 and col.data.shape[1] == 24
    got = col.data.cpu()
    want = ref[~bad] if handle == "skip" else ref
    assert got.shape[0] == want.shape[0]
    assert torch.equal(got[:, 17:], torch.zeros_like(got[:, 17:]))          # zero padding
    w = want.to(torch.bfloat16)
    same = (got[:, :17] == w) | (torch.isnan(got[:, :17].float()) & torch.isnan(w.float()))
    assert bool(same.all())
    if handle == "skip":
        kept = out.column_data("lab").data.cpu().long()
        assert torch.equal(kept, torch.nonzero(~bad).squeeze(1))


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["float32", "float64"])
def test_gpu_assemble_column_window_kernel(dtype):
    """assemble_cols_kernel (plain float / double columns, LDS-transposed windows) ==
    the generic gather kernel == a torch reference: several windows with a partial last
    one, a partial last row block, null masks and NaNs flagged per row."""
    import torch
    from orange3_spark_amd.ops import assemble as AS
    dev = torch.device("cuda", 0)
    dt = getattr(torch, dtype)
    g = torch.Generator().manual_seed(3)
    n, D = 1000 * 128 + 77, 203
    cols = [torch.randn(n, generator=g, dtype=dt) * 3 for _ in range(D)]
    cols[7][11] = float("nan")
    valid = torch.ones(n, dtype=torch.bool)
    valid[::331] = False
    srcs = [(c.to(dev), valid.to(dev) if j == 100 else None, 1) for j, c in enumerate(cols)]
    out, bad, nbad, d = AS.assemble_bf16(srcs, n, dev, path="cols")
    gen, gbad, gnbad, _ = AS.assemble_bf16(srcs, n, dev, path="generic")
    ref = torch.stack([c.float() for c in cols], 1)
    ref[:, 100] = torch.where(valid, ref[:, 100], torch.full_like(ref[:, 100], float("nan")))
    assert d == D and out.shape == gen.shape and out.shape[1] % 8 == 0
    assert torch.equal(out.view(torch.int16), gen.view(torch.int16))
    torch.testing.assert_close(out[:, :D].float().cpu(), ref.to(torch.bfloat16).float(), equal_nan=True)
    assert not out[:, D:].any()
    rb = torch.isnan(ref).any(1)
    assert torch.equal(bad.cpu().bool(), rb) and torch.equal(gbad, bad)
    assert int(nbad) == int(rb.sum()) == int(gnbad)


def test_native_string_packing_matches_arrow_buffers():
    """ops/text.py pack_strings (csrc/host_strings.cpp: length pass + threaded byte copy,
    no pyarrow) gives the Arrow (offsets, bytes, validity) of an ASCII column, and falls
    back to pyarrow for anything that is not a compact ASCII str."""
    from orange3_spark_amd.ops import text as TX
    rng = np.random.default_rng(3)
    words = np.array(["", "a", "Hello", "x y", "  lead", "tab\tsep"] + [f"w{i}" * (i % 7) for i in range(200)],
                     dtype=object)
    vals = words[rng.integers(0, len(words), 50_000)]
    vals[::97] = None
    offs, data, valid, ascii_ = TX.pack_strings(vals)
    o2, d2, v2 = TX.arrow_strings(vals)
    assert ascii_ is True and np.array_equal(offs, o2) and np.array_equal(data, d2) and np.array_equal(valid, v2)
    big = np.asarray(["z" * 1000] * 20_000, dtype=object)            # > 8 MB: the threaded copy
    offs, data, valid, _ = TX.pack_strings(big)
    assert valid is None and offs[-1] == 20_000_000 and bytes(data[-1000:]) == b"z" * 1000
    for odd in (["héllo", "a"], ["a", b"b"]):
        offs, data, valid, ascii_ = TX.pack_strings(np.asarray(odd, dtype=object))
        assert ascii_ is None


def test_native_string_packing_while_another_thread_mutates_the_column():
    """The native passes run with the GIL released (ADVICE/VERDICT r5): a second thread
    replacing elements of the caller's array (and dropping the old strings) while
    pack_strings runs must not change what is packed -- the passes work on a private
    snapshot -- and the result must be one consistent column."""
    import threading
    from orange3_spark_amd.ops import text as TX
    n = 20_000
    src = np.asarray(["a" * (600 + i % 50) for i in range(n)], dtype=object)      # > 8 MB: threaded copy
    stop = threading.Event()

    def mutate():
        k = 0
        while not stop.is_set():
            i = k % n
            src[i] = "b" * (1 + k % 3000)                  # frees the previous str (no other reference)
            k += 1
    th = threading.Thread(target=mutate)
    th.start()
    try:
        for _ in range(20):
            offs, data, valid, ascii_ = TX.pack_strings(src)
            assert ascii_ is True and valid is None and offs.shape == (n + 1,)
            lens = np.diff(offs)
            assert int(offs[-1]) == data.shape[0]
            for i in range(0, n, 997):                    # every string is wholly one version
                s = bytes(data[offs[i]:offs[i + 1]])
                assert s == b"a" * lens[i] or s == b"b" * lens[i]
    finally:
        stop.set()
        th.join()
