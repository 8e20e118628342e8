"""The native runtime pieces (radix indexer, block pool, xxh3) under
concurrent mutation + lookup, built standalone with AddressSanitizer +
UndefinedBehaviorSanitizer and with ThreadSanitizer."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "dynamo_exp_amd", "csrc", "tests", "stress_native.cpp")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
@pytest.mark.parametrize("san", ["address,undefined", "thread"])
def test_native_stress_under_sanitizer(tmp_path, san):
    exe = tmp_path / "stress"
    flags = ["-std=c++20", "-O1", "-g", f"-fsanitize={san}", "-fno-omit-frame-pointer"]
    if "undefined" in san:
        flags.append("-fno-sanitize-recover=undefined")
    subprocess.run(["g++", *flags, SRC, "-o", str(exe), "-lpthread"], check=True, timeout=300)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1", ASAN_OPTIONS="detect_leaks=1:halt_on_error=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    assert r.stdout.strip().endswith("ok")
