"""The resident services' release order, checked in the generated gfx950 code.

A service wave (kingdb_amd/csrc/service.h) writes a result with plain stores
and then the slot's done word; the host reads the bytes once it sees the word.
The release between them is an L2 write-back (buffer_wbl2) that must be
waited for (s_waitcnt vmcnt(0)) before the next store.  The compiler's
waitcnt pass dropped that wait whenever no load or store was outstanding (it
does not count the write-back), and the done word reached the host ahead of
the bytes: Gets in oracle/hook_mt.cc returned stale 64-byte pieces.  This
test compiles both service kernels' sources to assembly and checks that every
write-back is followed by a vmcnt(0) wait before any store, atomic or the
end of the program.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"
STORE = re.compile(r"(global_store|buffer_store|global_atomic|flat_store|flat_atomic|buffer_atomic|s_endpgm)")


def _asm(src, tmp_path):
    out = tmp_path / (os.path.basename(src) + ".s")
    cmd = [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-I" + os.path.join(ROOT, "include"),
           "-I" + os.path.join(ROOT, "kingdb_amd", "csrc"), "--cuda-device-only", "-S", src, "-o", str(out)]
    subprocess.run(cmd, check=True, capture_output=True, timeout=600)
    return out.read_text().split("\n")


def unwaited_writebacks(lines):
    """Line numbers of buffer_wbl2 not followed by a vmcnt(0) wait before the next store."""
    bad = []
    for i, line in enumerate(lines):
        if "buffer_wbl2" not in line:
            continue
        for nxt in lines[i + 1:]:
            t = nxt.strip()
            if t.startswith("s_waitcnt") and "vmcnt(0)" in t:
                break
            if STORE.match(t):
                bad.append(i + 1)
                break
    return bad


def test_checker_flags_the_bad_order():
    bad = ["\tbuffer_wbl2 sc0 sc1", "\ts_waitcnt lgkmcnt(0)", "\tglobal_store_dwordx2 v1, v[0:1], s[2:3] sc0 sc1"]
    good = ["\tbuffer_wbl2 sc0 sc1", "\ts_waitcnt vmcnt(0) lgkmcnt(0)", "\tglobal_store_dwordx2 v1, v[0:1], s[2:3]"]
    assert unwaited_writebacks(bad) == [1]
    assert unwaited_writebacks(good) == []


@pytest.mark.skipif(not shutil.which(HIPCC) and not os.path.exists(HIPCC), reason="hipcc absent")
@pytest.mark.parametrize("src", ["lz4_decompress.hip", "lz4_compress.hip"])
def test_service_writebacks_are_waited_for(src, tmp_path):
    lines = _asm(os.path.join(ROOT, "kingdb_amd", "csrc", src), tmp_path)
    assert any("buffer_wbl2" in line for line in lines), "no release in the service kernels?"
    assert unwaited_writebacks(lines) == []
