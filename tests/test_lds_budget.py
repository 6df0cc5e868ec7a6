"""LDS budgets the occupancy of the latency-bound kernels depends on (no GPU).

The hardware allocates a workgroup's LDS in 1 280-byte steps out of 160 KiB
(tools/probe/lds_occupancy.hip; every size probed on MI355X fits that rule,
profiles/r05/r05_occ.txt), so a kernel holds floor(163840 / ceil(lds / 1280) /
1280) one-wave workgroups per CU -- fewer than hipOccupancy... predicts for
sizes just over a step.  The compact byU32 compressor exists to hold all of a
batch's 2 560 1 MiB parts in one round (10 per CU); this test
reads the compiler's resource report and fails when its LDS grows past that.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"
STEP, TOTAL = 1280, 163840


def resident(lds: int) -> int:
    return TOTAL // (-(-lds // STEP) * STEP) if lds else 64


def test_step_rule_matches_probe():
    """The rule against the probe's measurements (r05_occ.txt)."""
    for lds, want in ((16384, 9), (16256, 9), (16000, 9), (15360, 10), (14400, 10), (20544, 7), (12800, 12),
                      (24576, 6), (6400, 25), (6656, 21), (7264, 21)):
        assert resident(lds) == want, lds


@pytest.mark.skipif(not shutil.which(HIPCC) and not os.path.exists(HIPCC), reason="hipcc absent")
def test_compact_kernel_holds_ten_per_cu():
    csrc = os.path.join(ROOT, "kingdb_amd", "csrc")
    r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-I" + os.path.join(ROOT, "include"),
                        "-I" + csrc, "-Rpass-analysis=kernel-resource-usage", "-c",
                        os.path.join(csrc, "lz4_compress.hip"), "-o", os.devnull],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    lds, name = {}, None
    for line in r.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            name = m.group(1)
        m = re.search(r"LDS Size \[bytes/block\]: (\d+)", line)
        if m and name:
            lds[name] = int(m.group(1))
    compact = [v for k, v in lds.items() if "big_compact_kernel" in k]
    assert compact, sorted(lds)
    assert all(resident(v) >= 10 for v in compact), compact


def groups_per_cu(lds: int) -> int:
    return TOTAL // (-(-lds // STEP) * STEP)


def decode_waves(region: int, regs_cap: int) -> tuple:
    """lz4_decompress.hip decode_waves: the waves per workgroup that put the
    most waves on a CU (ties: fewer per workgroup), and that count."""
    best, best_waves = 1, 0
    for w in range(1, 17):
        need = -(-region * w // STEP) * STEP
        if need > TOTAL:
            break
        waves = min(TOTAL // need * w, regs_cap)
        if waves > best_waves:
            best, best_waves = w, waves
    return best, best_waves


def test_multiwave_workgroups():
    """Several independent waves per workgroup pay the 1 280-byte step once per
    workgroup: ten 16 KiB compress waves fill exactly 160 KiB (10 per CU
    where one-wave workgroups hold 9), and the headline decoder's 7 264-byte
    waves (2 308-byte largest frame + the 4 KiB window: 6 512 bytes) go eight
    workgroups of three (24 per CU, the register limit, where one-wave ones
    hold 21)."""
    assert groups_per_cu(16384) * 1 == 9 and groups_per_cu(16384 * 10) * 10 == 10
    assert groups_per_cu(6512) == 21 and decode_waves(6512, 24) == (3, 24)
    assert decode_waves(7264, 24) == (11, 22)
    assert decode_waves(6400, 24) == (1, 24)        # one-wave workgroups already at the register cap
    assert decode_waves(8704, 24) == (1, 18)        # the mixed decoder's ring region: nothing to gain


@pytest.mark.skipif(not shutil.which(HIPCC) and not os.path.exists(HIPCC), reason="hipcc absent")
def test_ten_wave_compress_kernels_fit_160k():
    csrc = os.path.join(ROOT, "kingdb_amd", "csrc")
    r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-I" + os.path.join(ROOT, "include"),
                        "-I" + csrc, "-Rpass-analysis=kernel-resource-usage", "-c",
                        os.path.join(csrc, "lz4_compress.hip"), "-o", os.devnull],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    lds, name = {}, None
    for line in r.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            name = m.group(1)
        m = re.search(r"LDS Size \[bytes/block\]: (\d+)", line)
        if m and name:
            lds[name] = int(m.group(1))
    # lz4_compress_kernel<F, true, E, 10u> and lz4_compress_mixed_kernel<F, 10u>
    ten = {k: v for k, v in lds.items() if re.search(r"lz4_compress_kernelILb[01]ELb1ELj[012]ELj10E", k)
           or re.search(r"lz4_compress_mixed_kernelILb[01]ELj10E", k)}
    assert len(ten) == 6, sorted(lds)     # frame or not x batched or per-sequence emission, and mixed
    assert all(v == TOTAL for v in ten.values()), ten
