"""Lifetimes of the Python binding's views (no GPU): a Problem struct, a POINTER(Problem) and every
array view that SynthWindow / Graph hand out keep their owner alive, so reading them after the
owner's last reference is dropped (and a gc pass) reads the owner's memory, not freed memory.
Root cause it guards: gpurun_out/r04e (a test read the arrays of a SynthWindow that had already
been collected)."""
import gc
import weakref

import numpy as np

from _problem import OwnedProblem


def _window(og):
    return og.SynthWindow(5, 120, 600, seed=7)


def test_array_views_keep_the_window_alive(og):
    w = _window(og)
    ref = weakref.ref(w)
    expect = {k: getattr(w, k)().copy() for k in ("poses", "landmarks", "speed_biases", "imu_state", "extrinsics")}
    views = {k: getattr(w, k)() for k in expect}
    del w
    gc.collect()
    assert ref() is not None  # held by the views
    for k, v in views.items():
        assert np.array_equal(v, expect[k]), k
    views["poses"][0, 0] += 1.0  # still a live (writable) view of the window's memory
    assert views["poses"][0, 0] == expect["poses"][0, 0] + 1.0
    del views, v
    gc.collect()
    assert ref() is None  # and released once nothing refers to it


def test_problem_struct_and_pointer_keep_the_window_alive(og):
    w = _window(og)
    ref = weakref.ref(w)
    n_poses = w.problem.n_poses
    p0 = w.poses().copy()
    prob = w.problem
    ptr = _window(og).problem_ptr()  # a window only the pointer refers to
    del w
    gc.collect()
    assert ref() is not None
    assert prob.n_poses == n_poses
    assert np.array_equal(np.ctypeslib.as_array(prob.poses, shape=(n_poses, 7)), p0)
    # the deep copy the GPU tests make reads a problem whose window has no other reference
    cp = OwnedProblem.copy_of(ptr.contents)
    gc.collect()
    assert cp.poses.shape[1] == 7 and np.isfinite(cp.poses).all()
    del prob
    gc.collect()
    assert ref() is None
