"""Kernel variants and the product library.

The exact variants kept for A/B measurements (lane-counter scorer, inside-slab cull, 2-4 refine
producers, 2-3 frames per refine block, the chain prefetch, k_xrefine) and the measurement-only mode
that drops the chain's adds (wrong planes) are compiled only into the A/B build, libpitt_seg_ab.so.
The product library fixes every variant at its default and ignores their environment variables:
  * test_product_library_ignores_variant_knobs: with every knob set to a non-default value -- the
    chain-without-adds bit included -- the product library still returns the oracle's bits;
  * test_ab_library_variants_bit_exact: the variant parity modules (test_score_paths_gpu.py,
    test_xrefine_gpu.py) run under the A/B build in a child pytest, where the knobs do select the
    variants, so each variant stays exact."""
import os
import subprocess
import sys

import pytest

import pitt_object_table_segmentation_amd as pitt
from pitt_object_table_segmentation_amd import _lib
import test_plane_gpu as P

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
AB_LIB = os.path.join(ROOT, "pitt_object_table_segmentation_amd", "libpitt_seg_ab.so")
KNOBS = {"PITT_REFINE_MODE": "6", "PITT_LANE_SCORE": "1", "PITT_INSIDE_CULL": "1", "PITT_REFINE_PRODUCERS": "4",
         "PITT_REFINE_FRAMES": "3", "PITT_XREFINE": "2", "PITT_REFINE_DEBUG": "1"}


def test_product_library_ignores_variant_knobs():
    assert _lib.lib.pitt_build_flags() == 0, "the package must load the product library"
    old = {k: os.environ.get(k) for k in KNOBS}
    os.environ.update(KNOBS)
    try:
        c = pitt.Context(0)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    try:
        P.test_full_size_frames_bit_exact(c)
        P.test_ragged_batch_and_edge_frames(c)
        assert c.refine_stats() == (0, 0)  # k_xrefine never ran
    finally:
        c.close()


def test_ab_library_variants_bit_exact():
    assert os.path.exists(AB_LIB), "libpitt_seg_ab.so missing: __graft_entry__.build() builds it (make ab)"
    env = dict(os.environ, PITT_LIB_PATH=AB_LIB)
    cmd = [sys.executable, "-u", "-m", "pytest", "-x", "-q", "-m", "gpu", "-p", "no:cacheprovider",
           "--timeout", "300", "--timeout-method", "thread",
           os.path.join(ROOT, "tests", "test_score_paths_gpu.py"), os.path.join(ROOT, "tests", "test_xrefine_gpu.py")]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    tail = p.stdout[-3000:] + p.stderr[-2000:]
    assert p.returncode == 0, tail
    assert " passed" in p.stdout and " skipped" not in p.stdout.splitlines()[-1], tail
    print(p.stdout.splitlines()[-1])
