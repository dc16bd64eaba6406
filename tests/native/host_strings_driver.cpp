// Sanitizer driver for ops/csrc/host_strings.cpp (built by tests/test_native_sanitizers.py
// with -fsanitize=address,undefined, and with -fsanitize=thread around concurrent callers):
// embeds CPython, builds a column of compact-ASCII str / None / non-ASCII objects, and
// checks the length pass and the (threaded) byte copy against the strings themselves --
// with the GIL released during the calls, as ctypes.CDLL does in ops/text.py.
#include <Python.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <random>
#include <string>
#include <thread>
#include <vector>

extern "C" {
int64_t o3s_host_ascii_lengths(PyObject* const* objs, int64_t n, int64_t* offs, uint8_t* valid);
int o3s_host_ascii_pack(PyObject* const* objs, int64_t n, const int64_t* offs, uint8_t* out, int nthreads);
}

static int fails = 0;
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) { fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #c); ++fails; } \
  } while (0)

static void pack_and_check(const std::vector<PyObject*>& objs, const std::vector<std::string>& want,
                           const std::vector<bool>& none, int nthreads) {
  const int64_t n = (int64_t)objs.size();
  std::vector<int64_t> offs(n + 1);
  std::vector<uint8_t> valid(n);
  const int64_t tot = o3s_host_ascii_lengths(objs.data(), n, offs.data(), valid.data());
  CHECK(tot >= 0);
  if (tot < 0) return;
  std::vector<uint8_t> out((size_t)tot + 1);
  CHECK(o3s_host_ascii_pack(objs.data(), n, offs.data(), out.data(), nthreads) == 0);
  for (int64_t i = 0; i < n; ++i) {
    CHECK(valid[i] == (none[i] ? 0 : 1));
    const std::string got(reinterpret_cast<const char*>(out.data()) + offs[i], (size_t)(offs[i + 1] - offs[i]));
    CHECK(got == want[i]);
  }
}

int main(int argc, char** argv) {
  const bool threaded = argc > 1 && strcmp(argv[1], "threads") == 0;
  Py_Initialize();
  std::mt19937 rng(7);
  std::vector<PyObject*> objs;
  std::vector<std::string> want;
  std::vector<bool> none;
  for (int i = 0; i < 4000; ++i) {            // > 8 MB in total: the threaded copy path runs
    if (i % 97 == 0) {
      Py_INCREF(Py_None);
      objs.push_back(Py_None);
      want.emplace_back();
      none.push_back(true);
      continue;
    }
    std::string s((size_t)(rng() % 4000), 'a');
    for (auto& c : s) c = (char)(' ' + rng() % 95);
    objs.push_back(PyUnicode_FromStringAndSize(s.data(), (Py_ssize_t)s.size()));
    want.push_back(s);
    none.push_back(false);
  }
  PyThreadState* ts = PyEval_SaveThread();    // the calls run without the GIL (ctypes.CDLL)
  if (threaded) {
    std::vector<std::thread> th;
    for (int t = 0; t < 4; ++t) th.emplace_back([&, t] { pack_and_check(objs, want, none, 1 + t * 3); });
    for (auto& x : th) x.join();
  } else {
    pack_and_check(objs, want, none, 1);
    pack_and_check(objs, want, none, 8);
    std::vector<PyObject*> empty;
    int64_t off0 = -1;
    CHECK(o3s_host_ascii_lengths(empty.data(), 0, &off0, nullptr) == 0 && off0 == 0);
  }
  PyEval_RestoreThread(ts);
  // a non-ASCII string stops the length pass at its index (the caller falls back to pyarrow)
  PyObject* uni = PyUnicode_FromString("caf\xc3\xa9");
  std::vector<PyObject*> mixed = {objs[1], uni, objs[2]};
  std::vector<int64_t> offs(4);
  std::vector<uint8_t> valid(3);
  CHECK(o3s_host_ascii_lengths(mixed.data(), 3, offs.data(), valid.data()) == -2);
  Py_DECREF(uni);
  for (auto* o : objs) Py_DECREF(o);
  Py_FinalizeEx();
  if (fails) { fprintf(stderr, "%d checks failed\n", fails); return 1; }
  printf("host strings sanitizer driver ok (%s)\n", threaded ? "threads" : "serial");
  return 0;
}
