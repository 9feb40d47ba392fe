"""Regenerates tools/lab/fan_phases.patch from csrc/ + fan_lists.patch (the
fan-phase timers sit inside fanTraceD, so the patch is rebuilt whenever that
function changes): per-wave phase cycles and work counts of k_lidar_fan,
read back through mpenv_lab_fan (tools/kernel_lab.py prints them).

  python tools/kernel_lab.py build fanph --patch tools/lab/fan_lists.patch \
      --patch tools/lab/fan_phases.patch"""
import os
import re
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, "madrona-mp-env_amd", "csrc")


def sub(s, pat, repl, what):
    s2, n = re.subn(pat, repl, s, count=1, flags=re.S)
    if n != 1:
        sys.exit(f"make_fan_phases: anchor not found: {what}")
    return s2


def edit_geom(g):
    g = sub(g, r"(constexpr int kFanListCap = [^\n]*\n)", r"""\1
// lab overlay (tools/lab/fan_phases.patch): per-wave phase cycles and work
// counts of the forward-fan tasks, summed over the wave's tasks in `lab`
// (0 pre, 1 cull, 2 masks, 3 walk, 4 post, 5 tasks, 6 survivors, 7 entries
// walked, 8 entries tested, 9 lane tests; k_lidar_rear: 10 pre + traversal,
// 11 post, 12 tasks) and stored per wave at the end of the kernel (no
// atomics: contention would stretch what is measured).
constexpr int kLabFanWaves = 1 << 17, kLabFanK = 13;
static __device__ unsigned long long g_labFan[kLabFanWaves][kLabFanK];
""", "kFanListCap")
    g = sub(g, r"(mp::Vec3 &ray_o, mp::Vec3 &ray_d, float &t_out)\)\n\{\n    using namespace mp;\n",
            r"\1, uint64_t *lab)\n{\n    using namespace mp;\n    uint64_t lt = clock64();\n", "fanTraceD signature")
    g = sub(g, r"(    waveSync\(\);\n)(    const Vec3 oh0)",
            r"\1    { const uint64_t t = clock64(); lab[1] += t - lt; lt = t; }\n\2", "end of cull")
    g = sub(g, r"(    // 3\. walk[^\n]*\n(?:    //[^\n]*\n)*    mkRay\(ray_o, ray_d\);)",
            r"    { const uint64_t t = clock64(); lab[2] += t - lt; lt = t; }\n\1", "walk start")
    g = sub(g, r"(const bool act = [^\n]*\n)(\s*)if \(__ballot\(act\) == 0ull\) continue;",
            r"\1\2lab[7]++;\n\2if (__ballot(act) == 0ull) continue;\n\2lab[8]++;\n\2lab[9] += __popcll(__ballot(act));",
            "walk entry")
    g = sub(g, r"(    ch \+= \d+u;\n    \} while \(ch < count\);\n)(    t_out = t_best;)",
            r"    { const uint64_t t = clock64(); lab[3] += t - lt; lt = t; }\n\1    lab[6] += count;\n\2",
            "walk end")
    return g


def edit_kernels(k):
    k = sub(k, r"(    const uint32_t wave = __builtin_amdgcn_readfirstlane\(threadIdx\.x >> 6\);\n)"
               r"(    for \(int it = 0; it < iters; it\+\+\) \{\n)",
            r"\1    uint64_t lab[kLabFanK] = {};\n\2        const uint64_t lab_t0 = clock64();\n"
            r"        uint64_t lab_t2 = 0;\n", "lidar task loop")
    k = sub(k, r"(        if \(task >= ntasks\) break;\n)",
            r"\1        if (kMode == kLidarFan) lab[5]++;\n        if (kMode == kLidarRear) lab[12]++;\n", "task bound")
    k = sub(k, r"(bhit = bvhTraceRayT<[^;]*;\n        \}\n)",
            r"\1        if (kMode == kLidarRear) { lab_t2 = clock64(); lab[10] += lab_t2 - lab_t0; }\n", "rear trace")
    k = sub(k, r"(\n(\s*)fanTraceD\()", r"\n\2lab[0] += clock64() - lab_t0;\1", "fanTraceD call")
    k = sub(k, r"(ray_o, dir, tb)\);", r"\1, lab);", "fanTraceD args")
    k = sub(k, r"(bhit = __float_as_int\(tb\) != __float_as_int\(kFltMax\);\n)",
            r"\1            lab_t2 = clock64();\n", "after fanTraceD")
    k = sub(k, r"        if \(!valid\) continue;\n",
            "        if (!valid) { if (kMode != kLidarAll) lab[kMode == kLidarFan ? 4 : 11] += clock64() - lab_t2; "
            "continue; }\n", "valid")
    k = sub(k, r"(        \*dst = out;\n)(    \}\n\})",
            r"""\1        if (kMode != kLidarAll) lab[kMode == kLidarFan ? 4 : 11] += clock64() - lab_t2;
    }
    if (kMode != kLidarAll) {
        const uint32_t gw = blockIdx.x * kLidarWaves + wave;
        if ((threadIdx.x & 63) == 0 && gw < (uint32_t)kLabFanWaves)
            for (int q = kMode == kLidarFan ? 0 : 10; q < (kMode == kLidarFan ? 10 : kLabFanK); q++)
                g_labFan[gw][q] = lab[q];
    }
}""", "task end")
    k = sub(k, r"(static int check\(hipError_t e\) \{ return e == hipSuccess \? 0 : -1; \}\n)", r"""\1
// lab overlay: the per-wave sums of the last k_lidar_fan / k_lidar_rear
// launches, summed over waves into out[0..12] (the per-wave slots are cleared)
extern "C" int mpenv_lab_fan(uint64_t *out, int32_t n)
{
    static unsigned long long h[kLabFanWaves][kLabFanK];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_labFan), sizeof(h), 0, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    for (int q = 0; q < n && q < kLabFanK; q++) {
        unsigned long long s = 0;
        for (int w = 0; w < kLabFanWaves; w++) s += h[w][q];
        out[q] = s;
    }
    static unsigned long long zeros[kLabFanWaves][kLabFanK];
    return check(hipMemcpyToSymbol(HIP_SYMBOL(g_labFan), zeros, sizeof(zeros), 0, hipMemcpyHostToDevice));
}
""", "check()")
    return k


def main():
    with tempfile.TemporaryDirectory() as td:
        a, b = os.path.join(td, "a"), os.path.join(td, "b")
        shutil.copytree(CSRC, a)
        lists = os.path.join(ROOT, "tools", "lab", "fan_lists.patch")
        subprocess.run(["patch", "-s", "-p1", "-d", a, "-i", lists], check=True)
        shutil.copytree(a, b)
        for f, fn in (("geom_dev.h", edit_geom), ("kernels.hip", edit_kernels)):
            p = os.path.join(b, f)
            text = fn(open(p).read())
            open(p, "w").write(text)
        out = subprocess.run(["diff", "-ru", "a", "b"], cwd=td, capture_output=True, text=True).stdout
        out = re.sub(r"^(---|\+\+\+) (a|b)/(\S+)\t[^\n]*", r"\1 \2/\3", out, flags=re.M)
        open(os.path.join(ROOT, "tools", "lab", "fan_phases.patch"), "w").write(
            "# requires: fan_lists.patch\n" + out)
    print("wrote tools/lab/fan_phases.patch")


if __name__ == "__main__":
    main()
