"""Write a scene's lidar_tree.txt: the split ranks tools/trav_stats.cpp
TRAV_TUNE found for k_lidar's tree (its final "splitRank:" line), keyed to
the FNV-1a 64 of the scene's collisions.bin (scene.cpp readLidarTuning).

    python tools/write_lidar_tree.py SCENE_DIR "3:1 4:1 7:3 ..." [NOTE]
"""
import os
import sys


def fnv1a64(path):
    h = 1469598103934665603
    for b in open(path, "rb").read():
        h ^= b
        h = (h * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


def main():
    scene, ranks = sys.argv[1], sys.argv[2]
    note = sys.argv[3] if len(sys.argv) > 3 else ""
    pairs = []
    for tok in ranks.replace("splitRank:", "").split():
        hid, r = tok.split(":")
        pairs.append((int(hid), int(r)))
    lines = [
        "# k_lidar's tree for this scene: BVHBuildOpts::splitRank over scene.h",
        "# lidarBVHOpts() (heap index of a binary build node, root 1; rank of the",
        "# distinct SAH candidate split taken there) and collapseChoice (per 4-wide",
        "# node: which inner children its collapse opens).  Tuned by tools/trav_stats.cpp",
        "# TRAV_TUNE (k_lidar's lockstep model over recorded lidar fans), written",
        "# by tools/write_lidar_tree.py; ignored for any other collisions.bin.",
    ]
    if note:
        lines.append("# " + note)
    lines.append(f"collisions_fnv1a64 {fnv1a64(os.path.join(scene, 'collisions.bin')):016x}")
    # negative heap index: a collapse choice (BVHBuildOpts::collapseChoice)
    lines += [f"split {h} {r}" for h, r in sorted(pairs) if h > 0]
    lines += [f"collapse {-h} {r}" for h, r in sorted(pairs, key=lambda p: -p[0]) if h < 0]
    with open(os.path.join(scene, "lidar_tree.txt"), "w") as f:
        f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
