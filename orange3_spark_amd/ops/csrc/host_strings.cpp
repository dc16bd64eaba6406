// Host string packing (C ABI, libo3s_host.so): a numpy object column of Python str / None
// -> Arrow-style (offsets, bytes, validity) buffers for the device text kernels, without
// building a pyarrow array (pa.array walks every string through the codec machinery: ~150
// ms per million 300-byte documents, the whole cost of a device Tokenizer pass).
//
// Only compact ASCII strings are packed here (their characters ARE the UTF-8 bytes, stored
// right after the object header); any other object makes the length pass return a negative
// index and the caller falls back to pyarrow.  The objects are only read: no reference
// counts change and no Python API that could run Python code is called, so the calls run
// with the GIL released (ctypes.CDLL) while the caller keeps the column alive.
#include <Python.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <thread>
#include <vector>

extern "C" {

// Pass 1: offs[0..n] (bytes), valid[i] = 0 for None.  Returns the total byte count, or
// -(i + 1) for the first object i that is neither None nor a compact ASCII str.
__attribute__((visibility("default"))) int64_t o3s_host_ascii_lengths(PyObject* const* objs, int64_t n, int64_t* offs,
                                                                      uint8_t* valid) {
  int64_t tot = 0;
  offs[0] = 0;
  for (int64_t i = 0; i < n; ++i) {
    PyObject* o = objs[i];
    int64_t len = 0;
    if (o == Py_None) {
      valid[i] = 0;
    } else {
      if (!PyUnicode_Check(o) || !PyUnicode_IS_COMPACT_ASCII(o)) return -(i + 1);
      len = (int64_t)PyUnicode_GET_LENGTH(o);
      valid[i] = 1;
    }
    tot += len;
    offs[i + 1] = tot;
  }
  return tot;
}

// Pass 2: copy every string's bytes to out[offs[i] ..), rows split over nthreads threads.
__attribute__((visibility("default"))) int o3s_host_ascii_pack(PyObject* const* objs, int64_t n, const int64_t* offs,
                                                               uint8_t* out, int nthreads) {
  auto work = [&](int64_t a, int64_t b) {
    for (int64_t i = a; i < b; ++i) {
      const int64_t len = offs[i + 1] - offs[i];
      if (len) memcpy(out + offs[i], PyUnicode_DATA(objs[i]), (size_t)len);
    }
  };
  const int64_t total = offs[n];
  nthreads = std::max(1, std::min(nthreads, 64));
  if (nthreads == 1 || total < (8 << 20)) {
    work(0, n);
    return 0;
  }
  // split by bytes, not rows: row i starts thread t's range when offs[i] >= t * total / T
  std::vector<std::thread> th;
  int64_t a = 0;
  for (int t = 1; t <= nthreads; ++t) {
    const int64_t target = t == nthreads ? total : total / nthreads * t;
    const int64_t b = t == nthreads ? n : (int64_t)(std::lower_bound(offs, offs + n + 1, target) - offs);
    if (b > a) th.emplace_back(work, a, b);
    a = std::max(a, b);
  }
  for (auto& x : th) x.join();
  return 0;
}
}
