"""Dev probe: compare dumped last-known exports of two lab variants."""
import numpy as np
import os
import sys
a, b = sys.argv[1], sys.argv[2]
d = "gpurun_out"
for eid, row in ((13, 32), (17, 3)):
    x = np.fromfile(f"{d}/dump_{a}_{eid}.bin", np.float32).reshape(-1, 6, row)
    y = np.fromfile(f"{d}/dump_{b}_{eid}.bin", np.float32).reshape(-1, 6, row)
    diff = np.any(x != y, axis=2)
    ag, sl = np.nonzero(diff)
    print(eid, "rows differing", len(ag), "of", diff.size)
    alive = np.fromfile(f"{d}/dump_{a}_24.bin", np.float32)
    for i in range(min(12, len(ag))):
        g, k = ag[i], sl[i]
        print(" agent", g, "slot", k, "alive", alive[g], "base", x[g, k][:6], "var", y[g, k][:6])
    # pattern: agent index mod 64 (lane), mod 12 (world slot)
    if len(ag):
        print(" lanes", np.bincount(ag % 64, minlength=64)[:64].tolist())
        print(" slots", np.bincount(sl, minlength=6).tolist(), "i%12", np.bincount(ag % 12, minlength=12).tolist())
for f in os.listdir(d):
    if f.startswith("dump_"):
        os.remove(os.path.join(d, f))
