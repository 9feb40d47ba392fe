// Reduced k_obs mask loop ("k_obs mask read"): the opponent
// mask of pvpOpponentMasksSystem (sim.cpp:2562-2614) held in a float[6]
// array, stored, then read again after divergent work as
// `mask[k] == 1.f` (the float form k_obs avoids).  Host-checked on
// synthetic 2v2 worlds whose visibility bits put every lane in one of the
// three cases: own bit set, set only by the teammate (the early-exit loop
// below), or unset.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//         -fno-fast-math tools/repro_obs_mask.hip -o gpurun_out/repro_obs_mask
//   ./gpurun_out/repro_obs_mask      (exit 0 = float and bits forms agree)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int kMax = 6;

template <bool kFloat>
__global__ void __launch_bounds__(256) k_mask(const float *alive, const uint8_t *vm, const float *firedT,
                                             const float *other, float *masks, float *knows, int T, int A)
{
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= A) return;
    const int N = 2 * T;
    const int w = g / N, i = g - w * N, team = i / T, off = i - team * T, g0 = w * N;
    const bool self_alive = alive[g] != 0.f;
    float mask[kMax];
    for (int k = 0; k < kMax; k++) {
        mask[k] = 0.f;
        if (!self_alive || k >= T) continue;
        const int go = g0 + (team ^ 1) * T + k;
        if (alive[go] == 0.f) continue;
        bool can_see = (vm[g] >> k) & 1;
        for (int t = 0; t < T - 1 && !can_see; t++) {
            const int gt = g0 + team * T + (t < off ? t : t + 1);
            if ((vm[gt] >> k) & 1) can_see = true;
        }
        if (can_see) mask[k] = 1.f;
        if (firedT[go] >= 0) mask[k] = 1.f;
    }
    for (int k = 0; k < kMax; k++) masks[g * kMax + k] = mask[k];
    uint32_t bits = 0;
    for (int k = 0; k < kMax; k++) bits |= (mask[k] == 1.f ? 1u : 0u) << k;
    // divergent work between the masks and their second read, as the
    // teammate rows are in k_obs
    float acc[kMax];
    for (int k = 0; k < kMax; k++) {
        acc[k] = 0.f;
        if (k < T && alive[g0 + team * T + (k % T)] != 0.f) {
            for (int j = 0; j < 8; j++) acc[k] += other[(g * kMax + k) * 8 + j] * float(j + 1);
        }
    }
    for (int k = 0; k < kMax; k++) {
        float v = -1.f;
        if (k < T && alive[g0 + (team ^ 1) * T + k] != 0.f) {
            const bool kn = kFloat ? mask[k] == 1.f : ((bits >> k) & 1u) != 0;
            v = (kn ? 1.f : 0.f) + 0.f * acc[k];
        }
        knows[g * kMax + k] = v;
    }
}

int main()
{
    const int T = 2, N = 4, W = 4096, A = W * N;
    std::vector<float> alive(A, 1.f), fired(A, -3.4028235e38f), other((size_t)A * kMax * 8, 0.5f);
    std::vector<uint8_t> vm(A);
    uint32_t s = 12345u;
    for (int g = 0; g < A; g++) {
        s = s * 1664525u + 1013904223u;
        vm[g] = (uint8_t)((s >> 16) & 3u);
    }
    float *dA, *dF, *dO, *dM, *dK;
    uint8_t *dV;
    hipMalloc(&dA, A * 4); hipMalloc(&dF, A * 4); hipMalloc(&dO, other.size() * 4);
    hipMalloc(&dM, (size_t)A * kMax * 4); hipMalloc(&dK, (size_t)A * kMax * 4); hipMalloc(&dV, A);
    hipMemcpy(dA, alive.data(), A * 4, hipMemcpyHostToDevice);
    hipMemcpy(dF, fired.data(), A * 4, hipMemcpyHostToDevice);
    hipMemcpy(dO, other.data(), other.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dV, vm.data(), A, hipMemcpyHostToDevice);
    int bad_total = 0;
    for (int form = 0; form < 2; form++) {
        if (form) k_mask<true><<<(A + 255) / 256, 256>>>(dA, dV, dF, dO, dM, dK, T, A);
        else k_mask<false><<<(A + 255) / 256, 256>>>(dA, dV, dF, dO, dM, dK, T, A);
        if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 2; }
        std::vector<float> m((size_t)A * kMax), kn((size_t)A * kMax);
        hipMemcpy(m.data(), dM, m.size() * 4, hipMemcpyDeviceToHost);
        hipMemcpy(kn.data(), dK, kn.size() * 4, hipMemcpyDeviceToHost);
        int bad = 0, bad_mate = 0, bad_own = 0;
        for (int g = 0; g < A; g++) {
            const int w = g / N, i = g - w * N, team = i / T, off = i - team * T;
            const int mate = w * N + team * T + (1 - off);
            for (int k = 0; k < T; k++) {
                const bool own = (vm[g] >> k) & 1, viaMate = (vm[mate] >> k) & 1;
                const float want = (own || viaMate) ? 1.f : 0.f;
                if (m[(size_t)g * kMax + k] != want) { printf("form %d: stored mask wrong at %d/%d\n", form, g, k); return 3; }
                if (kn[(size_t)g * kMax + k] != want) {
                    bad++;
                    if (own) bad_own++; else bad_mate++;
                }
            }
        }
        printf("%s form: %d wrong knows of %d (own bit set: %d, set by the teammate loop: %d)\n",
               form ? "float" : "bits", bad, A * T, bad_own, bad_mate);
        bad_total += bad;
    }
    return bad_total ? 1 : 0;
}
