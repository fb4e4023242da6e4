"""The diagnostic builds stay compilable (CPU: hipcc cross-compiles gfx950).

The product never compiles them: csrc/rt_diag.h turns every hook into
nothing unless RT_STAMPS / RT_PHASE_TWICE / RT_GTIMES / RT_BVH_CHECK is set,
and tools/stamps_run.py, tools/phase_lanes.sh, tools/gtimes_run.py and the
BVH check build set them.  A hook that no longer compiles would only show
up on the GPU box; this catches it here, one device-only compile per
translation unit with the hooks of both kernels' builds switched on."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "bwidman-raytracer_amd", "csrc")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
FLAGS = ["-O1", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off", "-fno-slp-vectorize",
         "-fno-unroll-loops", "--cuda-device-only", "-c", "-o", os.devnull]


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
@pytest.mark.parametrize("tu,defines", [
    ("rt_kernels.hip", ["-DRT_WAVES_PER_EU=6", "-DRT_STAMPS", "-DRT_BRANCH_STATS", "-DRT_GTIMES", "-DRT_PHASE_TWICE=4"]),
    ("rt_kernels.hip", ["-DRT_WAVES_PER_EU=6", "-DRT_PHASE_TWICE=3"]),
    ("rt_kernels_bvh.hip", ["-DRT_WAVES_PER_EU=4", "-DRT_STAMPS", "-DRT_GTIMES", "-DRT_BVH_CHECK"]),
])
def test_diagnostic_build_compiles(tu, defines):
    r = subprocess.run([HIPCC] + FLAGS + defines + [os.path.join(CSRC, tu)], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
