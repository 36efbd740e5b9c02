"""The sweep-form bucket sum's speed rests on its instruction schedule: each
burst's loads issued together, then waited on with counted vmcnt(N).  One
compiler choice regrouped the register tiles' adds into load -> vmcnt(0) ->
add chains (117-224 full drains per chunk, 8.3 instead of 6.5 ms at 8 buckets;
profiles/r01b/sweep_ab.txt).  This compiles the product kernel translation units to gfx950
assembly (no GPU needed) and fails if that comes back."""
import os
import re
import shutil
import subprocess

import pytest

from conftest import REPO

HIPCC = "/opt/rocm/bin/hipcc"


@pytest.fixture(scope="module")
def asm(tmp_path_factory):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not installed")
    # both translation units over gp_kernels.hpp: gp_reduce.hip launches the
    # plain forms (bucket sums, row plans), gp_unplanned.hip the GATED ones
    # (the unplanned calls' steady state); each instantiates its own copy
    # (compiled side by side)
    d = tmp_path_factory.mktemp("asm")
    tus = ("gp_unplanned", "gp_reduce")
    procs = [subprocess.Popen([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-I",
                               os.path.join(REPO, "include"), "--cuda-device-only", "-S", "-o", str(d / f"{tu}.s"),
                               os.path.join(REPO, "geeps_amd", "csrc", f"{tu}.hip")],
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, cwd=str(d)) for tu in tus]
    for p in procs:
        _, err = p.communicate()
        assert p.returncode == 0, err.decode()[-2000:]
    return "".join((d / f"{tu}.s").read_text() for tu in tus)


def _kernel(asm, pattern):
    m = re.search(rf"^({pattern}\S*):", asm, re.M)
    assert m, pattern
    body = asm[m.end():asm.index(".Lfunc_end", m.end())]
    return body


# (buckets, register tiles, tiles per burst, zero-input, 4-KiB block-strides
# per tile): every production instantiation (gp_kernels.hpp: SweepShape's
# 96-MiB chunks, the 64-MiB chunks after them, the zero-input form)
SWEEP_SHAPES = ([(1, 14, 8, 0, 4)] + [(nb, 7, 1, 0, 8) for nb in range(2, 9)]
                + [(nb, 6, 4, 0, 4) for nb in range(3, 9)] + [(1, 6, 4, 1, 4)])


@pytest.mark.parametrize("nb,rt,tg,zin,u", SWEEP_SHAPES)
def test_sweep_kernel_keeps_burst_schedule(asm, nb, rt, tg, zin, u):
    # (the last template argument: GATED = false, the form every launch but
    # the unplanned calls' steady state uses; GATED = true differs only by the
    # gate test before this body)
    body = _kernel(asm, rf"_ZN12_GLOBAL__N_123bucket_sum_sweep_kernelILi{nb}ELi{rt}ELi{tg}ELb{zin}ELi{u}ELb0EE")
    loads = len(re.findall(r"global_load_dwordx4", body))
    full_drains = len(re.findall(r"s_waitcnt vmcnt\(0\)", body))
    streams = nb if zin else nb + 1
    lds_tiles = 40 // u  # 160 KiB of LDS in tiles of u * 4 KiB
    # streams x (LDS + register) tiles x u block-strides, all dwordx4
    assert loads == streams * (lds_tiles + rt) * u
    # production: at most one full drain per burst; the regressed schedule
    # drained once per 16-KiB tile or more (117-224 at 8 buckets)
    bursts = streams * (lds_tiles + rt) // tg
    assert full_drains <= bursts, f"{full_drains} full vmcnt(0) drains: the burst schedule regressed"
    # each burst's loads are issued together: some wait leaves the rest of a
    # burst (u * tg - 1 loads) in flight
    counts = [int(n) for n in re.findall(r"s_waitcnt vmcnt\((\d+)\)", body)]
    assert max(counts) >= u * tg - 1, f"at most {max(counts)} loads in flight: bursts split"
    assert "scratch_" not in body and "buffer_store_dword" not in body  # no spills


def test_wave_kernels_fit_their_occupancy(asm):
    """The scatter / gather wave-map kernels keep 3-4 waves per SIMD: the
    limit-straddle path must not index register arrays at run time (that cost
    86-91 more VGPRs and halved the resident blocks; profiles/r02)."""
    for op, max_vgpr in ((0, 168), (1, 128), (3, 128)):  # add, gather, init at 128-float rows
        # <f4, OP, 32 lanes, 8 rows, flat, MAP 0 (the production tile map), not gated>
        pat = rf"_ZN12_GLOBAL__N_115row_wave_kernelIDv4_fLi{op}ELi32ELi8ELi0ELi0ELb0EEE"
        name = re.search(rf"^({pat}\S*):", asm, re.M).group(1)
        n = int(re.search(rf"\.set {re.escape(name)}\.num_vgpr, (\d+)", asm).group(1))
        assert n <= max_vgpr, (op, n)


@pytest.mark.parametrize("rt,tg,zin", [(14, 8, 0), (6, 4, 1), (6, 4, 0)])
def test_gated_sweep_kernel_keeps_burst_schedule(asm, rt, tg, zin):
    """The GATED = true forms (the unplanned calls' steady state, gp_unplanned.hip
    "Device-built plans") run the gate test, then the same body: the same
    loads, and no more full drains than the plain form."""
    plain = _kernel(asm, rf"_ZN12_GLOBAL__N_123bucket_sum_sweep_kernelILi1ELi{rt}ELi{tg}ELb{zin}ELi4ELb0EE")
    gated = _kernel(asm, rf"_ZN12_GLOBAL__N_123bucket_sum_sweep_kernelILi1ELi{rt}ELi{tg}ELb{zin}ELi4ELb1EE")
    for body in (plain, gated):
        assert "scratch_" not in body
    assert gated.count("global_load_dwordx4") == plain.count("global_load_dwordx4")
    drains = lambda b: len(re.findall(r"s_waitcnt vmcnt\(0\)", b))
    assert drains(gated) <= drains(plain) + 1
