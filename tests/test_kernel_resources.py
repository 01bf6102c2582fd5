"""Register/scratch audit of the release library's gfx950 kernels, read from the code-object metadata
of the built .so (no GPU).  A kernel with scratch (private segment) bytes spills registers to memory
or keeps a runtime-indexed register array there; both cost per-lane memory round trips on the step's
critical path (round 4 found the chain stage-A kernel at 240 B/lane and seg_fft at 64 B/lane)."""
import os
import re
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import kernel_resources as KR  # noqa: E402

LIB = os.path.join(ROOT, "sclmd_amd", "_lib", "libhipgle.so")


@pytest.fixture(scope="module")
def rows():
    if not os.path.exists(LIB):
        pytest.skip("release library not built (make)")
    if not os.path.exists(KR.READELF):
        pytest.skip("llvm-readelf missing")
    return KR.kernel_resources(LIB)


def test_every_source_has_gfx950_kernels(rows):
    names = " ".join(r["name"] for r in rows)
    for k in ("chain_kernel", "cgemm_kernel", "seg_fft_kernel", "contract_kernel", "philox_kernel", "fpot_kernel"):
        assert k in names, k


def test_no_scratch(rows):
    bad = [(r["name"], r.get("private_segment_fixed_size"), r.get("vgpr_spill_count"))
           for r in rows if r.get("private_segment_fixed_size", 0) or r.get("vgpr_spill_count", 0)]
    assert not bad, bad


def test_register_budgets(rows):
    # the step kernels' occupancy rests on these budgets: chain stage kernels
    # with 4-wave groups at one DOF column tile stay within 128 VGPRs (2 waves / SIMD plus the
    # background far-field work), 8-wave groups within 128 (launch bound 512 threads)
    checked = 0
    for r in rows:
        n = r["name"]
        if "chain_kernel" in n and re.search(r"ILi\dELi(4ELi1|8ELi\d)E", n):
            assert r["vgpr_count"] <= 128, (n, r["vgpr_count"])
            checked += 1
    assert checked == 18  # stages 0-5 (5: the composed stage with one-column VALU products) x (4, 1), (8, 1), (8, 2)


def test_demangler_optional():
    assert shutil.which("c++filt") is None or KR._demangle(["_Z3foov"]) == ["foo()"]
