"""Where the workgroups of a CU-masked stream run (tools/cu_mask_probe.hip): for the masks
aimet_amd.calibration builds (side stream with k CUs per XCD, and its complement), count the distinct
CUs (XCC_ID, SE, SH, CU from HW_ID) each XCD contributes. Expect k per XCD for the side mask and
32 - k for the complement if the mask layout spreads over the XCDs as intended."""
import collections
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from aimet_amd.calibration import side_cu_mask  # noqa: E402

lib = ctypes.CDLL(os.path.join(REPO, "tools", "cu_mask_probe.so"))
BLOCKS = 4096


def where(words):
    arr = (ctypes.c_uint32 * max(1, len(words)))(*(words or [0]))
    out = (ctypes.c_uint32 * (2 * BLOCKS))()
    rc = lib.probe_where(arr, len(words), BLOCKS, out)
    assert rc == 0, rc
    per_xcd = collections.defaultdict(set)
    for b in range(BLOCKS):
        xcc, hw = out[2 * b] & 0xF, out[2 * b + 1]
        per_xcd[xcc].add(((hw >> 13) & 7, (hw >> 12) & 1, (hw >> 8) & 0xF))
    return {x: len(v) for x, v in sorted(per_xcd.items())}


res = {"full": where([])}
for k in (1, 2, 4):
    side = side_cu_mask(256, k)
    main = [0xFFFFFFFF & ~w for w in side]
    res["side_%d_per_xcd" % k] = where(side)
    res["main_complement_%d" % k] = where(main)
print(json.dumps(res), flush=True)
