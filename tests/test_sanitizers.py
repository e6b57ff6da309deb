"""Host sanitizers: AddressSanitizer + UndefinedBehaviorSanitizer over the host code.

* include/mim_detect.hpp (the clustering / margin / merge / metrics stages after the matcher,
  TestsDetector.cpp:111-248, metrics.cpp) through tests/cpp/test_detect.cpp: the whole
  test_detect_host.py suite runs against an ASan/UBSan build of the driver too (its `driver`
  fixture is parametrized), so every case there is sanitizer-checked.
* The CPU restatement (oracle/mim_oracle.c, oracle/sift_oracle.c) through tests/cpp/oracle_san.c:
  built plain and sanitized, both must exit cleanly with identical output.
GPU AddressSanitizer is not available on the GPU pool, so the device code is not covered here."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g"]
SAN_ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")


def _build_oracle_driver(exe, sanitize):
    src = [os.path.join(ROOT, "oracle", "mim_oracle.c"), os.path.join(ROOT, "oracle", "sift_oracle.c"),
           os.path.join(ROOT, "tests", "cpp", "oracle_san.c")]
    flags = ["-O1", "-ffp-contract=off", "-fno-fast-math", "-std=c11", "-D_GNU_SOURCE", "-Wall"]
    subprocess.check_call(["gcc", *flags, *(SAN if sanitize else []), *src, "-o", exe, "-lm", "-lpthread"])


def test_oracle_under_asan_ubsan(tmp_path):
    plain, san = str(tmp_path / "plain"), str(tmp_path / "san")
    _build_oracle_driver(plain, False)
    _build_oracle_driver(san, True)
    a = subprocess.run([plain], capture_output=True, text=True, timeout=300)
    b = subprocess.run([san], capture_output=True, text=True, timeout=600, env=SAN_ENV)
    assert a.returncode == 0, a.stderr[-3000:]
    assert b.returncode == 0, b.stderr[-6000:]
    assert "runtime error" not in b.stderr and "AddressSanitizer" not in b.stderr, b.stderr[-6000:]
    assert a.stdout == b.stdout and a.stdout.endswith("OK\n"), (a.stdout, b.stdout)
    out = dict(line.split(" ", 1) for line in a.stdout.splitlines() if " " in line)
    assert int(out["knn"].split()[-1]) > 20  # the planted matches survive the ratio test
    assert out["collinear"] in ("0", "1")  # n == 4: runKernel alone, no checkSubset (ptsetreg.cpp)
    assert out["sift-tiny"] == "0" and int(out["sift-cap"]) > 3

