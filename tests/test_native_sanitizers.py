"""Host-side sanitizer runs of the native C++ runtime (SURVEY §5 "race detection /
sanitizers"): the host library sources are compiled together with a driver under
AddressSanitizer + UndefinedBehaviorSanitizer, and under ThreadSanitizer with concurrent
callers, then run on the CPU.  (GPU-side sanitizers are not available on the MI355X pool;
kernel races are covered by the bitwise determinism tests of the HIP kernels.)"""
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "orange3_spark_amd" / "ops" / "csrc"
DRIVER = ROOT / "tests" / "native" / "host_sanitize_driver.cpp"
SOURCES = [CSRC / "host_text.cpp", CSRC / "host_pav.cpp", DRIVER]


def _cxx():
    return shutil.which("g++") or shutil.which("clang++")


STRINGS = [CSRC / "host_strings.cpp", ROOT / "tests" / "native" / "host_strings_driver.cpp"]


def _py_build():
    """(include dir, link flags) of the embedded CPython the strings driver runs."""
    import sysconfig
    inc = sysconfig.get_paths()["include"]
    libdir = sysconfig.get_config_var("LIBDIR")
    ver = sysconfig.get_config_var("LDVERSION") or sysconfig.get_config_var("VERSION")
    return inc, [f"-L{libdir}", f"-Wl,-rpath,{libdir}", f"-lpython{ver}"]


def _build_and_run(tmp_path, flags, args=(), sources=SOURCES, extra=(), leaks=True):
    exe = tmp_path / "driver"
    cmd = [_cxx(), "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", *flags, "-I", str(CSRC),
           *map(str, sources), "-o", str(exe), "-lpthread", *extra]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    r = subprocess.run([str(exe), *args], capture_output=True, text=True, timeout=120,
                       env={"ASAN_OPTIONS": f"detect_leaks={int(leaks)}:abort_on_error=1",
                            "UBSAN_OPTIONS": "halt_on_error=1", "TSAN_OPTIONS": "halt_on_error=1"})
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def _strings_build_args():
    inc, link = _py_build()
    if not (Path(inc) / "Python.h").exists():
        pytest.skip("Python headers not installed")
    return ["-I", inc], link


@pytest.mark.skipif(_cxx() is None, reason="no host C++ compiler")
def test_host_strings_asan_ubsan(tmp_path):
    """csrc/host_strings.cpp (the GIL-released str packer) under ASan + UBSan, embedded in
    CPython (interpreter leaks at exit are CPython's, so leak checking is off here)."""
    inc, link = _strings_build_args()
    out = _build_and_run(tmp_path, ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", *inc],
                         sources=STRINGS, extra=link, leaks=False)
    assert "strings sanitizer driver ok (serial)" in out


@pytest.mark.skipif(_cxx() is None, reason="no host C++ compiler")
def test_host_strings_tsan_concurrent_callers(tmp_path):
    inc, link = _strings_build_args()
    try:
        out = _build_and_run(tmp_path, ["-fsanitize=thread", *inc], ["threads"], sources=STRINGS, extra=link)
    except subprocess.CalledProcessError as e:          # toolchain without libtsan
        pytest.skip(f"ThreadSanitizer unavailable: {e.stderr[-200:]}")
    assert "strings sanitizer driver ok (threads)" in out


@pytest.mark.skipif(_cxx() is None, reason="no host C++ compiler")
def test_host_runtime_asan_ubsan(tmp_path):
    out = _build_and_run(tmp_path, ["-fsanitize=address,undefined", "-fno-sanitize-recover=all"])
    assert "ok" in out


@pytest.mark.skipif(_cxx() is None, reason="no host C++ compiler")
def test_host_runtime_tsan_concurrent_callers(tmp_path):
    try:
        out = _build_and_run(tmp_path, ["-fsanitize=thread"], ["threads"])
    except subprocess.CalledProcessError as e:          # toolchain without libtsan
        pytest.skip(f"ThreadSanitizer unavailable: {e.stderr[-200:]}")
    assert "threads" in out
