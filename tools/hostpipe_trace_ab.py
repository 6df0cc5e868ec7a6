"""Does tracing perturb the host-inclusive compress?
Untraced compress/decompress runs, then profile() tracing all span kinds,
only the kernels, only the copies, then untraced again; prints wall times.

    python tools/hostpipe_trace_ab.py
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import kingdb_amd as K
    from kingdb_amd.hostpipe import HostPipeline
    K.set_device(0)
    n, size = 1 << 20, 4096
    b = K.DeviceBatch.g1_long_sizes(np.full(n, size, np.uint32))
    hp = HostPipeline(n, size)
    hp.h_raw.np[:] = b.src.download(n * size)
    hp.compress(), hp.decompress()
    out = {"untraced": [(round(hp.compress() * 1e3, 2), round(hp.decompress() * 1e3, 2)) for _ in range(3)]}
    for name, kinds in (("all", None), ("kernel", ["kernel"]), ("h2d", ["h2d"]), ("d2h", ["d2h"]), ("all2", None)):
        p = hp.profile(kinds)
        out[name] = {ph: p[ph]["wall_ms"] for ph in ("compress", "decompress")}
    out["untraced_after"] = [(round(hp.compress() * 1e3, 2), round(hp.decompress() * 1e3, 2)) for _ in range(3)]
    out["ok"] = bool(np.array_equal(hp.h_out.np, hp.h_raw.np))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
