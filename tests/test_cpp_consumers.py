"""The boundary from C and C++ callers (not only ctypes): tests/cpp/abi_consumer.c is compiled as
C99 with -pedantic against include/okvisgpu.h, tests/cpp/facade_test.cpp as C++17 against the
::ceres::Problem-subset facade include/okvisgpu_problem.hpp, both with the host compilers only and
linked to libokvisgpu.so. CPU: build + bookkeeping / error paths. GPU: solves through both."""
import os
import subprocess

import pytest

from _paths import REPO

CPP = os.path.join(REPO, "tests", "cpp")


@pytest.fixture(scope="module")
def consumers():
    # built by __graft_entry__.build(); rebuilt here only if missing or stale (make is a no-op otherwise)
    r = subprocess.run(["make", "-C", CPP], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    return CPP


def _run(consumers, exe, mode):
    return subprocess.run([os.path.join(consumers, exe), mode], capture_output=True, text=True, timeout=240)


def test_c_consumer_cpu(consumers):
    r = _run(consumers, "abi_consumer", "cpu")
    assert r.returncode == 0, r.stderr
    assert "abi_consumer cpu ok: ABI 6, 10 poses / 500 landmarks / 4000 observations" in r.stdout


def test_facade_cpu(consumers):
    r = _run(consumers, "facade_test", "cpu")
    assert r.returncode == 0, r.stdout + r.stderr
    assert "facade_test cpu ok" in r.stdout


def test_header_is_plain_c():
    """The C ABI header compiles as C99 and as C++11 on its own (-pedantic -Werror)."""
    src = "#include \"okvisgpu.h\"\nint main(void) { okvisgpu_options o; okvisgpu_problem p; (void)o; (void)p; return 0; }\n"
    for cc, std, ext in (("gcc", "-std=c99", ".c"), ("g++", "-std=c++11", ".cpp")):
        path = os.path.join("/tmp", "okvisgpu_hdr" + ext)
        with open(path, "w") as f:
            f.write(src)
        r = subprocess.run([cc, std, "-pedantic", "-Wall", "-Werror", "-fsyntax-only", "-I",
                            os.path.join(REPO, "include"), path], capture_output=True, text=True)
        assert r.returncode == 0, r.stderr


@pytest.mark.gpu
def test_c_consumer_gpu(consumers, og, oracle):
    import json
    r = _run(consumers, "abi_consumer", "gpu")
    assert r.returncode == 0, r.stderr
    d = json.loads(r.stdout.strip().splitlines()[-1])
    w = og.SynthWindow(10, 500, 4000, seed=20251015)
    so = oracle.solve(w.problem_ptr(), og.default_options(max_num_iterations=10))
    assert d["num_iterations"] == so["num_iterations"] and d["termination"] == so["termination_type"]
    assert abs(d["final_cost"] - so["final_cost"]) <= 1e-7 * so["final_cost"]
    assert max(abs(a - b) for a, b in zip(d["pose9"], w.poses()[9, :3])) <= 1e-6


@pytest.mark.gpu
def test_facade_gpu(consumers):
    r = _run(consumers, "facade_test", "gpu")
    assert r.returncode == 0, r.stdout + r.stderr
    assert "facade_test gpu ok" in r.stdout
