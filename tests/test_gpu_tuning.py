"""libvhx reads no environment for its schedule or its correctness: scheduling knobs go through
vhx_set_tuning, and the two diagnostics that change behaviour are compile-time variant builds only.

* every former VHX_* knob set to a hostile value before the library loads changes nothing: the default frame still
  equals the golden digests, and tree writes stay ordered against frames in flight;
* the negative control: the VHX_UNORDERED_WRITES=1 variant build (built by __graft_entry__.build(), never the shipped
  library) fails the ordering test, so that test detects a missing ordering;
* vhx_set_tuning refuses malformed specs and leaves the schedule unchanged.
"""
import os
import subprocess
import sys

import pytest

import voxelhex_amd as vhx
from voxelhex_amd import _build

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# the environment knobs libvhx read up to round 3, each with a value that would have changed the schedule, its
# ordering or its diagnostics
HOSTILE = {"VHX_UNORDERED_WRITES": "1", "VHX_DEBUG_PASSES": "1", "VHX_BUDGETS": "1,2,3", "VHX_ADAPTIVE": "0",
           "VHX_RPW": "1,1,1", "VHX_TW": "1", "VHX_XCDG": "7", "VHX_RESUME": "0", "VHX_SAVE_FROM": "2",
           "VHX_QBLOCK": "64", "VHX_QWAVES": "3", "VHX_QWAVESM": "5", "VHX_QWAVES0": "9", "VHX_QXCD": "1",
           "VHX_SPARSE": "64,64", "VHX_QORDER": "m4096z", "VHX_SPLIT": "1", "VHX_SPLIT_WAIT": "1",
           "VHX_SPLIT_DIAG": "3", "VHX_SPLIT_TUNE": "1,2,1,1", "VHX_QXCD_ALL": "1", "VHX_MIP_GENERIC": "1",
           "VHX_MIP_THREADS": "1", "VHX_MIP_TIMING": "1"}


def _pytest_child(tests, env, timeout=600):
    return subprocess.run([sys.executable, "-u", "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider", *tests],
                          cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)


def test_hostile_environment_changes_nothing():
    env = dict(os.environ, **HOSTILE)
    r = _pytest_child(["tests/test_gpu_golden.py::test_gpu_frame_matches_golden[c2_256_bd4_1920x1080]",
                       "tests/test_gpu_ordering.py::test_ranged_writes_between_frames_in_flight"], env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    assert "2 passed" in r.stdout, r.stdout[-2000:]


def test_unordered_variant_build_is_detected():
    lib = _build.UNORDERED_LIB
    assert os.path.exists(lib), "variant build missing: run __graft_entry__.build()"
    env = dict(os.environ, VHX_LIB=lib)
    r = _pytest_child(["tests/test_gpu_ordering.py::test_ranged_writes_between_frames_in_flight"], env)
    assert r.returncode != 0 and "differs at" in r.stdout, \
        "the ordering test passed without the ordering: " + r.stdout[-3000:] + r.stderr[-2000:]


def test_set_tuning_validates_and_applies():
    rt = vhx.Raytracer(0)
    try:
        rt.set_tuning("budgets=16,128;qorder=32r")
        assert rt.pass_budgets() == ((16, 128), "fixed")
        for bad in ("nokey=1", "budgets=3,2", "qblock=100", "qorder=12", "rpw=65", "split_tune=3,2,1,1", "adaptive",
                    "budgets=1;bogus=2", "sparse=1,x", "qsort=100", "qsort=4096", "qsort=768", "stage_slots=0",
                    "stage_slots=5", "tail=2", "tail_min=0", "tail_rpw=0", "tail_rpw=65", "tail_prio=4",
                    "tail_cap=2000000", "qwpc_idle=0", "qwpc_busy=65", "sbudget=x", "qwaves0=0"):
            with pytest.raises(Exception):
                rt.set_tuning(bad)
            assert rt.pass_budgets() == ((16, 128), "fixed"), bad  # a refused spec changes nothing
        # the round-6 keys that leave the schedule alone
        rt.set_tuning("stage_slots=4;tail=1;tail_min=300;tail_rpw=8;tail_prio=2;tail_cap=512;sbudget=48;qwaves0=2048")
        assert rt.pass_budgets() == ((16, 128), "fixed")
        rt.set_tuning({"adaptive": 1})
        rt.set_tuning("qwpc_idle=8;qwpc_busy=3")  # per-schedule figures: the choice stays adaptive
        rt.set_tuning("budgets=")
        assert rt.pass_budgets()[0] == ()
    finally:
        rt.close()
