"""Build-time checks of the HIP kernel sources (CPU only: hipcc cross-compiles gfx950)."""
import os
import shutil

import pytest

from dynamo_exp_amd import build_native

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


@pytest.mark.skipif(not shutil.which(HIPCC) and not os.path.exists(HIPCC), reason="hipcc not available")
@pytest.mark.timeout(900)
def test_kernels_pass_llvm_machine_verifier():
    """Every kernel source's gfx950 machine code passes -verify-machineinstrs.  Round 5's decode-attention merge
    change tripped a ROCm 7.2 sub-register liveness miscompile that only showed on the GPU as wrong G = 1 outputs;
    the verifier names it at compile time ("No live subrange at use")."""
    bad = build_native.verify_kernels(jobs=min(8, os.cpu_count() or 1))
    assert not bad, "machine verifier rejected:\n" + "\n".join(f"{k}:\n{v}" for k, v in bad.items())
