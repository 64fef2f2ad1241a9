"""C-ABI boundary checks that need no GPU: the library loads, exports exactly the entry points
include/okvisgpu.h declares, reports errors instead of crashing without a device, and its
default options are Ceres' Solver::Options defaults plus the okvis settings."""
import ctypes as C
import os
import re
import shutil
import subprocess

import pytest

from _paths import REPO

HEADER = os.path.join(REPO, "include", "okvisgpu.h")


def _declared():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    txt = re.sub(r"//[^\n]*", "", txt)
    return sorted(set(re.findall(r"\b(okvisgpu_\w+)\s*\(", txt)))


def test_header_declares_the_python_symbol_list(og):
    assert _declared() == sorted(og.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol(og):
    lib = og.lib()
    for name in _declared():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", og.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (okvisgpu_\w+)", out))
    assert exported == set(_declared())


def test_library_is_gfx950_code(og, tmp_path):
    # (--offloading writes the extracted bundles next to its input: run it on a copy)
    lib = tmp_path / "lib.so"
    shutil.copyfile(og.LIB_PATH, lib)
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", str(lib)],
                         capture_output=True, text=True, cwd=tmp_path)
    if out.returncode != 0:
        pytest.skip("llvm-objdump --offloading unavailable")
    assert "gfx950" in out.stdout + out.stderr


def test_abi_version_and_phase_names(og):
    lib = og.lib()
    assert lib.okvisgpu_abi_version() >= 1
    names = [lib.okvisgpu_phase_name(i) for i in range(og.N_PHASES)]
    assert all(n for n in names) and len(set(names)) == og.N_PHASES
    assert lib.okvisgpu_phase_name(og.N_PHASES) in (None, b"")


def test_default_options_are_ceres_defaults(og):
    o = og.default_options()
    # ceres::Solver::Options defaults (types.h / solver.h of Ceres >= 2.1) as used by okvis, which
    # sets only DOGLEG, DENSE_SCHUR, max_num_iterations and num_threads (ViGraph.cpp:248-249,1854)
    assert o.trust_region_strategy == 0 and o.linear_solver == 0  # OKVISGPU_DOGLEG, OKVISGPU_DENSE_SCHUR
    assert o.function_tolerance == 1e-6 and o.gradient_tolerance == 1e-10 and o.parameter_tolerance == 1e-8
    assert o.initial_trust_region_radius == 1e4 and o.max_trust_region_radius == 1e16
    assert o.min_trust_region_radius == 1e-32 and o.min_relative_decrease == 1e-3
    assert o.min_lm_diagonal == 1e-6 and o.max_lm_diagonal == 1e32
    assert o.max_num_consecutive_invalid_steps == 5 and o.jacobi_scaling == 1


def test_no_device_is_an_error_not_a_crash(og):
    if og.device_count() > 0:
        pytest.skip("a GPU is visible")
    h = C.c_void_p()
    rc = og.lib().okvisgpu_ctx_create(0, C.byref(h))
    assert rc != 0 and not h.value


def test_null_arguments_are_rejected(og):
    lib = og.lib()
    assert lib.okvisgpu_solve(None, None, None) != 0
    assert lib.okvisgpu_set_problems(None, None, 0) != 0
    assert lib.okvisgpu_synth_create(None, None) != 0


def test_struct_layouts_match_the_header(og, tmp_path):
    """The ctypes structs mirror include/okvisgpu.h (sizes and the offsets of the fields added in
    ABI 6: okvisgpu_problem.host_loss, the okvisgpu_summary timing fields, okvisgpu_loss)."""
    if not shutil.which("gcc"):
        pytest.skip("gcc unavailable")
    fields = {"okvisgpu_problem": ["host_loss", "host_evaluate", "host_cauchy", "n_host", "extrinsics_constant"],
              "okvisgpu_summary": ["final_mu", "preprocessor_time_s", "minimizer_time_s", "postprocessor_time_s",
                                   "linear_solver_time_s", "residual_evaluation_time_s",
                                   "jacobian_evaluation_time_s", "step_time_s"],
              "okvisgpu_loss": ["kind", "reserved", "a", "b"],
              "okvisgpu_options": ["cholesky_schedule", "verbose"]}
    src = ["#include <stdio.h>", "#include <stddef.h>", '#include "okvisgpu.h"', "int main(void) {"]
    for t, fs in fields.items():
        src.append(f'  printf("{t} %zu\\n", sizeof({t}));')
        for f in fs:
            src.append(f'  printf("{t}.{f} %zu\\n", offsetof({t}, {f}));')
    src += ["  return 0;", "}"]
    c = tmp_path / "layout.c"
    c.write_text("\n".join(src))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c99", "-I", os.path.join(REPO, "include"), str(c), "-o", str(exe)], check=True)
    got = dict(line.split() for line in subprocess.run([str(exe)], capture_output=True, text=True).stdout.splitlines())
    py = {"okvisgpu_problem": og.Problem, "okvisgpu_summary": og.Summary, "okvisgpu_loss": og.Loss,
          "okvisgpu_options": og.Options}
    for t, cls in py.items():
        assert int(got[t]) == C.sizeof(cls), t
        for f in fields[t]:
            assert int(got[f"{t}.{f}"]) == getattr(cls, f).offset, (t, f)
    assert og.LOSS_DTYPE.itemsize == C.sizeof(og.Loss)


@pytest.mark.gpu
def test_summary_timings(og):
    """okvisgpu_summary's Ceres Summary timing fields (FullReport at ViGraph.cpp:1887-1889):
    wall clock of preprocessing / minimizer / postprocessing always; with options.verbose the
    iterations run as timed eager launches and the linear-solver / residual / Jacobian evaluation
    device times are filled (else -1), and the solve's bits are those of the graph-launched solve."""
    res = []
    for verbose in (0, 1):
        w = og.SynthWindow(10, 500, 4000, seed=20251015)
        ctx = og.Context(0)
        try:
            ctx.set_problems([w.problem])
            o = og.default_options(max_num_iterations=6, function_tolerance=0.0, gradient_tolerance=0.0,
                                   parameter_tolerance=0.0, verbose=verbose)
            s = ctx.solve(o)[0]
        finally:
            ctx.close()
        res.append((s, w.poses().copy()))
    (s0, x0), (s1, x1) = res
    assert s0["num_iterations"] == s1["num_iterations"] == 6 and s0["final_cost"] == s1["final_cost"]
    import numpy as np
    assert np.array_equal(x0, x1)
    for s in (s0, s1):
        parts = s["preprocessor_time_s"] + s["minimizer_time_s"] + s["postprocessor_time_s"]
        assert min(s["preprocessor_time_s"], s["minimizer_time_s"], s["postprocessor_time_s"]) >= 0.0
        assert parts <= s["total_time_s"] * 1.0001 + 1e-6, s
    assert s0["linear_solver_time_s"] == s0["residual_evaluation_time_s"] == s0["jacobian_evaluation_time_s"] == -1.0
    dev = [s1[k] for k in ("linear_solver_time_s", "residual_evaluation_time_s", "jacobian_evaluation_time_s",
                           "step_time_s")]
    assert all(t > 0.0 for t in dev), s1
    assert sum(dev) <= s1["minimizer_time_s"] * 1.0001, s1
