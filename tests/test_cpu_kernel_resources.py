"""Resource guard on the built library (CPU, no GPU): every gfx950 kernel of the in-tree objects keeps its data in
registers and LDS -- no scratch (private segment) memory, LDS within a CU's 160 KiB -- read from the code
objects' metadata (tools/kernel_resources.py).  Scratch in a streaming kernel is an HBM round trip per spilled
value: the burst epilogue with torch CPU's restated sqrt once spilled its register-held tiles (528 bytes per lane)
and lost 9 points of HBM bandwidth before the build raised LLVM's pragma-unroll threshold (nvflare_amd/_build.py)."""

import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import kernel_resources as kr  # noqa: E402


@pytest.fixture(scope="module")
def ks():
    if not os.path.isdir(kr.OBJ) or not os.path.exists(os.path.join(kr.LLVM, "clang-offload-bundler")):
        pytest.skip("library objects or the ROCm LLVM tools are absent")
    res = kr.all_kernels()
    if not res:
        pytest.skip("no kernel metadata found")
    return res


def test_no_kernel_uses_scratch(ks):
    bad = [(k["object"], k["name"], k["scratch"]) for k in ks if k["scratch"]]
    assert not bad, bad[:10]


def test_lds_and_registers_fit_a_cu(ks):
    assert all(k["lds"] <= 160 * 1024 for k in ks)
    assert all(k["vgpr"] <= 512 for k in ks)  # .vgpr_count: arch and accumulation VGPRs together on gfx950
    names = [k["name"] for k in ks]
    for needed in ("fedavg_tiles_burst_f32x4", "fedavg_tiles_epi_burst_f32x4", "fedavg_sqrt_f32",
                   "fedavg_tiles_epi_dma_f32x4", "fedavg_tiles_epi_split_f32x4"):
        assert any(needed in n for n in names), needed


def test_two_wave_per_simd_kernels_fit_256_registers(ks):
    """The 512-thread kernels (two waves per SIMD, one block per CU: the split-epilogue form, the LDS-DMA form at W = 8)
    get 256 registers per wave, arch and accumulation VGPRs together; more would not fit the block on a CU."""
    wide = [k for k in ks if "fedavg_tiles_epi_split_f32x4" in k["name"] or
            ("fedavg_tiles_epi_dma_f32x4" in k["name"] and "Li8EEEv" in k["name"])]  # mangled: W = 8 is the last arg
    assert wide, "no 512-thread kernel found"
    bad = [(k["name"], k["vgpr"], k["agpr"]) for k in wide if k["vgpr"] > 256]
    assert not bad, bad[:5]


@pytest.mark.timeout(600)
def test_no_result_copy_before_a_join_blocks_exec_restore():
    """No kernel of the product library holds the miscompile round 6 met in the LDS-DMA fused form (tools/
    check_join_copies.py, fedavg_arith.h wave_any): a VALU write in a divergent branch's join block placed before the
    block's exec restore, to a register written nowhere else -- the lanes that skipped the branch lose the value.  The
    rare-case recomputes branch on a wave-uniform condition since; the library built before that had 18 such kernels."""
    import check_join_copies as cj

    lib = os.path.join(ROOT, "nvflare_amd", "lib", "libnvflare_amd_fedavg.so")
    if not os.path.exists(lib) or not os.path.exists(os.path.join(cj.LLVM, "llvm-objdump")):
        pytest.skip("the library or the ROCm LLVM tools are absent")
    n, flagged = cj.scan_so(lib, jobs=min(8, os.cpu_count() or 1))
    assert n > 1000
    assert not flagged, [(k[:100], f[:2]) for k, f in flagged[:5]]
