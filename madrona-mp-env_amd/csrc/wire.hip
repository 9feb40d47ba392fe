// wire.hip — the learner exchange's compact wire format.
//
// mpenv_wire_pack turns one step of a shard's trainInterface outputs
// (mgr.cpp:2383-2431, 3,924 B per agent as exported) into a message of
// ~477 B per agent + 160 B per world; mpenv_wire_unpack, on the learner,
// rebuilds every output bit for bit into a shadow manager of the same
// configuration:
//   * lidar as the f32 depth of each ray plus its class in two bit-planes
//     (none / wall / teammate / opponent), 340 B per agent instead of 1,280:
//     pvpLidarSystem writes (min(t, maxDist), wall, teammate, opponent) or
//     (-1, 0, 0, 0) (sim.cpp:3324-3506), so the class decides the three
//     one-hot channels;
//   * the observation rows (self, teammates, opponents, positions, masks,
//     filters) are not shipped: the message carries the agent and world
//     state they are computed from and the shadow runs the same k_obs on it,
//     so the rows come out of the same device code on the same inputs;
//   * the last-known rows are the one piece of history k_obs reads: the
//     shadow keeps its own copy, clears a world's rows when that world's
//     episode counter moves (resetPersistentEntities is the only other
//     writer, level_gen.cpp:330-370) and k_obs updates them as on the
//     sender; a keyframe message carries them once (the first message of an
//     exchange, which may start mid-episode);
//   * small integer fields are packed into one word; the pack kernel flags
//     any value outside its packed range (or a lidar ray off the pattern
//     above) in the header and unpack then refuses the message.
// Columns are structure-of-arrays blocks, 256-B aligned, so both kernels
// read and write coalesced rows (thread = agent, ray or world).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstddef>
#include <cstdint>

#include "engine.h"
#include "mpenv_core.h"

namespace mpenv {

using namespace mp;

constexpr uint32_t kWireMagic = 0x3157504du; // "MPW1"
constexpr uint32_t kWireVersion = 1;
constexpr uint32_t kWireKeyframe = 1u, kWireOverflow = 2u;
// error word bits (mpenv_wire_error)
constexpr uint32_t kWireErrRefused = MPENV_WIRE_ERR_REFUSED, kWireErrDesync = MPENV_WIRE_ERR_DESYNC;

// agent f32 columns, agent i32 columns, world i32 columns (order = wire order)
#define MP_WIRE_AF(X) \
    X(px) X(py) X(pz) X(vx) X(vy) X(vz) X(rw) X(rx) X(ry) X(rz) X(ayaw) X(apitch) X(dyv) X(dpv) X(firedT)
#define MP_WIRE_AI(X) X(transRem) X(wasShot) X(autohealSteps)
#define MP_WIRE_WI(X) \
    X(curStep) X(filtMatched0) X(filtMatched1) X(curZone) X(controlling) X(contested) X(captured) \
    X(stepsUntilPoint) X(zoneSteps) X(episodeCounter)
#define MP_COUNT(n) +1
constexpr int kWireAF = 0 MP_WIRE_AF(MP_COUNT);
constexpr int kWireAI = 0 MP_WIRE_AI(MP_COUNT);
constexpr int kWireWI = 0 MP_WIRE_WI(MP_COUNT);
#undef MP_COUNT

struct WireHeader {
    uint32_t magic, version, flags, worldOffset;
    int32_t W, N, T, pad;
    int64_t A, bytes;
    uint32_t reserved[8];
};
static_assert(sizeof(WireHeader) == 80, "wire header");

struct WireLayout {
    int64_t af[kWireAF], hp, alive, reward; // f32 [A]
    int64_t ai[kWireAI], done, mag;         // i32 [A] (mag: [A][2])
    int64_t packed;                         // u32 [A]: curPose | tgtPose << 8 | weapon << 16 | flags << 24
    int64_t vis;                            // u8 [A]
    int64_t coefs;                          // f32 [A][9]
    int64_t depth;                          // f32 [A * 80]
    int64_t plane[2];                       // u32 [ceil(A * 80 / 32)]
    int64_t wi[kWireWI], match;             // i32 [W], [W][30]
    int64_t lkObs, lkPos;                   // keyframes: f32 [A][6][32], [A][6][3]
    int64_t total;
};

__host__ __device__ inline WireLayout wireLayout(int64_t A, int64_t W, bool keyframe)
{
    WireLayout L {};
    int64_t off = 256; // header
    auto take = [&](int64_t bytes) {
        const int64_t o = off;
        off += (bytes + 255) / 256 * 256;
        return o;
    };
    for (int k = 0; k < kWireAF; k++) L.af[k] = take(A * 4);
    L.hp = take(A * 4);
    L.alive = take(A * 4);
    L.reward = take(A * 4);
    for (int k = 0; k < kWireAI; k++) L.ai[k] = take(A * 4);
    L.done = take(A * 4);
    L.mag = take(A * 8);
    L.packed = take(A * 4);
    L.vis = take(A);
    L.coefs = take(A * 36);
    L.depth = take(A * kLidarRays * 4);
    const int64_t words = (A * kLidarRays + 31) / 32;
    L.plane[0] = take(words * 4);
    L.plane[1] = take(words * 4);
    for (int k = 0; k < kWireWI; k++) L.wi[k] = take(W * 4);
    L.match = take(W * 120);
    L.lkObs = keyframe ? take(A * 6 * kOtherObs * 4) : -1;
    L.lkPos = keyframe ? take(A * 18 * 4) : -1;
    L.total = off;
    return L;
}

// ------------------------------------------------------------------ pack
// One launch, four block ranges (round 4's three launches: ~40 us of the
// ~105 us pack were the agent and world kernels' latency and the boundaries):
//   lidar   thread = ray (agent * 80 + ray, forward rays first): the depth,
//           and the class in two bit-planes (one ballot per plane per 64 rays);
//   agents  thread = agent: state columns (and, for a keyframe, the
//           last-known rows);
//   worlds  thread = world: world columns; thread 0 the header;
//   match   thread = 16 bytes of the [W][30] episode results, copied flat.
// The header's flags word is zeroed before the launch (launchWirePack) and
// every writer ORs its bits in, so no block's order matters.
struct WirePackGrid {
    uint32_t agents, worlds, match, total; // first block of each range (lidar = 0), then the total
};

__host__ __device__ inline WirePackGrid wirePackGrid(int64_t A, int64_t W)
{
    auto blocks = [](int64_t n) { return (uint32_t)((n + 255) / 256); };
    WirePackGrid G;
    G.agents = blocks(A * kLidarRays);
    G.worlds = G.agents + blocks(A);
    G.match = G.worlds + blocks(W);
    G.total = G.match + blocks((W * 120 + 15) / 16);
    return G;
}

__global__ void __launch_bounds__(256) k_wire_pack(DevState S, char *dst, WireLayout L, WirePackGrid G,
                                                   uint32_t worldOffset)
{
    const uint32_t b = blockIdx.x;
    uint32_t *hflags = &reinterpret_cast<WireHeader *>(dst)->flags;
    if (b < G.agents) {
        const int64_t r = (int64_t)b * 256 + threadIdx.x;
        const int64_t nr = S.A * kLidarRays;
        uint32_t c = 0;
        bool ok = true;
        if (r < nr) {
            const int64_t g = r / kLidarRays;
            const int k = (int)(r - g * kLidarRays);
            const float4 v = k < kFwdRays ? reinterpret_cast<const float4 *>(S.fwdLidar)[g * kFwdRays + k]
                                          : reinterpret_cast<const float4 *>(S.rearLidar)[g * kRearRays + k - kFwdRays];
            reinterpret_cast<float *>(dst + L.depth)[r] = v.x;
            const uint32_t y = __float_as_uint(v.y), z = __float_as_uint(v.z), w = __float_as_uint(v.w);
            const uint32_t one = 0x3f800000u;
            if (y == one && z == 0u && w == 0u) c = 1;
            else if (y == 0u && z == one && w == 0u) c = 2;
            else if (y == 0u && z == 0u && w == one) c = 3;
            else ok = y == 0u && z == 0u && w == 0u && __float_as_uint(v.x) == 0xbf800000u; // (-1, 0, 0, 0)
        }
        const uint64_t b0 = __ballot(c & 1u), b1 = __ballot(c >> 1);
        const int lane = threadIdx.x & 63;
        const int64_t word = (r - lane) / 32; // first of the wave's two words
        const int64_t words = (nr + 31) / 32;
        if (lane < 4) {
            const int p = lane >> 1, h = lane & 1;
            const uint64_t bb = p ? b1 : b0;
            if (word + h < words) reinterpret_cast<uint32_t *>(dst + L.plane[p])[word + h] = (uint32_t)(bb >> (32 * h));
        }
        if (!ok) atomicOr(hflags, kWireOverflow);
    } else if (b < G.worlds) {
        const int64_t g = (int64_t)(b - G.agents) * 256 + threadIdx.x;
        if (g >= S.A) return;
        // every load first, then the stores (loads issued after stores wait
        // for the stores' acknowledgements: gfx9 retires them in order)
        float af[kWireAF];
        int32_t ai[kWireAI];
        int k = 0;
#define MP_GET_F(n) af[k++] = S.n[g];
        MP_WIRE_AF(MP_GET_F)
#undef MP_GET_F
        k = 0;
#define MP_GET_I(n) ai[k++] = S.n[g];
        MP_WIRE_AI(MP_GET_I)
#undef MP_GET_I
        const float hp = S.hp[g], alive = S.alive[g], reward = S.reward[g];
        const int32_t done = S.done[g];
        const int2 mag = make_int2(S.magazine[2 * g], S.magazine[2 * g + 1]);
        const int32_t cp = S.curPose[g], tp = S.tgtPose[g], wp = S.weapon[g], fl = S.flags[g];
        const uint8_t vis = S.visMask[g];
        float coef[9];
        for (int c = 0; c < 9; c++) coef[c] = S.rewardCoefs[g * 9 + c];
        for (k = 0; k < kWireAF; k++) reinterpret_cast<float *>(dst + L.af[k])[g] = af[k];
        for (k = 0; k < kWireAI; k++) reinterpret_cast<int32_t *>(dst + L.ai[k])[g] = ai[k];
        reinterpret_cast<float *>(dst + L.hp)[g] = hp;
        reinterpret_cast<float *>(dst + L.alive)[g] = alive;
        reinterpret_cast<float *>(dst + L.reward)[g] = reward;
        reinterpret_cast<int32_t *>(dst + L.done)[g] = done;
        reinterpret_cast<int2 *>(dst + L.mag)[g] = mag;
        const bool fits = ((uint32_t)cp | (uint32_t)tp | (uint32_t)wp | (uint32_t)fl) < 256u;
        reinterpret_cast<uint32_t *>(dst + L.packed)[g] =
            (uint32_t)cp | ((uint32_t)tp << 8) | ((uint32_t)wp << 16) | ((uint32_t)fl << 24);
        reinterpret_cast<uint8_t *>(dst + L.vis)[g] = vis;
        for (int c = 0; c < 9; c++) reinterpret_cast<float *>(dst + L.coefs)[g * 9 + c] = coef[c];
        if (L.lkObs >= 0) {
            const float4 *src = reinterpret_cast<const float4 *>(S.lkObs + g * 6 * kOtherObs);
            float4 *o = reinterpret_cast<float4 *>(dst + L.lkObs) + g * 6 * kOtherObs / 4;
            for (int q = 0; q < 6 * kOtherObs / 4; q++) o[q] = src[q];
            for (int q = 0; q < 18; q++) reinterpret_cast<float *>(dst + L.lkPos)[g * 18 + q] = S.lkPos[g * 18 + q];
        }
        if (!fits) atomicOr(hflags, kWireOverflow);
    } else if (b < G.match) {
        const int64_t w = (int64_t)(b - G.worlds) * 256 + threadIdx.x;
        if (w == 0) {
            WireHeader *h = reinterpret_cast<WireHeader *>(dst);
            h->magic = kWireMagic;
            h->version = kWireVersion;
            h->worldOffset = worldOffset;
            h->W = S.W; h->N = S.N; h->T = S.T; h->pad = 0;
            h->A = S.A;
            h->bytes = L.total;
            if (L.lkObs >= 0) atomicOr(hflags, kWireKeyframe);
        }
        if (w >= S.W) return;
        int32_t wv[kWireWI];
        int k = 0;
#define MP_GET_W(n) wv[k++] = S.n[w];
        MP_WIRE_WI(MP_GET_W)
#undef MP_GET_W
        for (k = 0; k < kWireWI; k++) reinterpret_cast<int32_t *>(dst + L.wi[k])[w] = wv[k];
    } else {
        const int64_t i = (int64_t)(b - G.match) * 256 + threadIdx.x;
        const int64_t bytes = S.W * 120;
        if (i * 16 >= bytes) return;
        if (i * 16 + 16 <= bytes) {
            reinterpret_cast<uint4 *>(dst + L.match)[i] = reinterpret_cast<const uint4 *>(S.matchResult)[i];
        } else {
            for (int64_t o = i * 16; o < bytes; o += 4)
                reinterpret_cast<int32_t *>(dst + L.match)[o / 4] = S.matchResult[o / 4];
        }
    }
}

// ---------------------------------------------------------------- unpack
// Every unpack kernel checks the header first: a message for another
// configuration or shard (world offset), of the other kind (keyframe or not),
// or one the pack kernels flagged is not unpacked, and raises both error
// bits.  A refused message leaves the shadow out of sync (the next plain
// messages build on history it missed: last-known rows, episode counters),
// so the desync bit is sticky: later plain messages are refused too (refused
// bit again), and only a keyframe, which carries that history, is unpacked
// and clears it.  k_obs_wire, launched after k_wire_unpack on the same
// stream, skips a shadow whose desync bit is set (DevState::obsGate), so its
// rows are never rebuilt from stale state.  Senders send a keyframe every
// `keyframe_every` messages (mpenv_dist.LearnerWire), so a shadow recovers.
__device__ __forceinline__ bool wireOk(const DevState &S, const char *src, const WireLayout &L, uint32_t *err,
                                       uint32_t worldOffset)
{
    const WireHeader *h = reinterpret_cast<const WireHeader *>(src);
    const bool keyframe = L.lkObs >= 0;
    const bool hdr = h->magic == kWireMagic && h->version == kWireVersion && h->W == S.W && h->N == S.N &&
                     h->A == S.A && h->bytes == L.total && h->worldOffset == worldOffset &&
                     !(h->flags & kWireOverflow) && ((h->flags & kWireKeyframe) != 0) == keyframe;
    const bool ok = hdr && (keyframe || !(*(volatile uint32_t *)err & kWireErrDesync));
    if (!ok && blockIdx.x == 0 && threadIdx.x == 0) atomicOr(err, hdr ? kWireErrRefused : kWireErrRefused | kWireErrDesync);
    return ok;
}

// The learner's rebuild of one message (launchWireUnpack), two launches:
//   k_wire_unpack, one launch in four block ranges --
//     lidar   thread = 4 rays 256 apart (1,024 consecutive rays per block):
//             the depth and the class bits of each, a float4 of f32 lidar out
//             per ray -- every load and store instruction unit-stride;
//     agents  thread = agent: the per-agent outputs that are state columns
//             (hp, alive, reward, done, magazine, reward coefficients) and,
//             for a keyframe, the last-known rows;
//     worlds  thread = world: the message's episode counters, kept for the
//             next message's reset test (double-buffered: next != prev);
//     match   thread = 16 bytes of the [W][30] episode results, copied flat;
//   k_obs_wire (kernels.hip) -- the observation rows, read straight from the
//     message's state columns (the shadow's own state columns are not
//     written: round 5 stored ~90 B per agent there and k_obs read them
//     back), with the last-known clear of a reset world folded in.
struct WireUnpackGrid {
    uint32_t lidar, agents, worlds, match; // first block of each range (lidar = 0), then the total
    uint32_t total;
};

__host__ __device__ inline WireUnpackGrid wireUnpackGrid(int64_t A, int64_t W)
{
    auto blocks = [](int64_t n) { return (uint32_t)((n + 255) / 256); };
    WireUnpackGrid G;
    G.lidar = 0;
    G.agents = (uint32_t)((A * kLidarRays + 1023) / 1024);
    G.worlds = G.agents + blocks(A);
    G.match = G.worlds + blocks(W);
    G.total = G.match + blocks((W * 120 + 15) / 16);
    return G;
}

__global__ void __launch_bounds__(256) k_wire_unpack(DevState S, const char *src, WireLayout L, WireUnpackGrid G,
                                                     uint32_t *err, uint32_t worldOffset, int32_t *epNext)
{
    if (!wireOk(S, src, L, err, worldOffset)) return;
    const uint32_t b = blockIdx.x;
    // an accepted keyframe resynchronises the shadow (keyframes ignore the
    // desync bit, so no block's decision depends on when this lands)
    if (L.lkObs >= 0 && b == 0 && threadIdx.x == 0) atomicAnd(err, ~kWireErrDesync);
    if (b < G.agents) {
        // 1,024 consecutive rays per block, ray base + 256 j + thread: each
        // load and store instruction is unit-stride (a 64-B run per lane made
        // every store instruction 16-B pieces at a 64-B stride)
        const int64_t nr = S.A * kLidarRays;
        const int64_t r0 = (int64_t)b * 1024 + threadIdx.x;
        float d[4];
        uint32_t cl[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int64_t r = r0 + 256 * j;
            d[j] = 0.f;
            cl[j] = 0;
            if (r < nr) {
                d[j] = reinterpret_cast<const float *>(src + L.depth)[r];
                const uint32_t sh = (uint32_t)(r & 31);
                cl[j] = ((reinterpret_cast<const uint32_t *>(src + L.plane[0])[r >> 5] >> sh) & 1u) |
                        (((reinterpret_cast<const uint32_t *>(src + L.plane[1])[r >> 5] >> sh) & 1u) << 1);
            }
        }
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int64_t r = r0 + 256 * j;
            if (r >= nr) break;
            const int64_t g = r / kLidarRays;
            const int k = (int)(r - g * kLidarRays);
            float4 *dst = k < kFwdRays ? reinterpret_cast<float4 *>(S.fwdLidar) + g * kFwdRays + k
                                       : reinterpret_cast<float4 *>(S.rearLidar) + g * kRearRays + (k - kFwdRays);
            const uint32_t c = cl[j];
            *dst = make_float4(d[j], c == 1 ? 1.f : 0.f, c == 2 ? 1.f : 0.f, c == 3 ? 1.f : 0.f);
        }
    } else if (b < G.worlds) {
        const int64_t g = (int64_t)(b - G.agents) * 256 + threadIdx.x;
        if (g >= S.A) return;
        const float hp = reinterpret_cast<const float *>(src + L.hp)[g];
        const float alive = reinterpret_cast<const float *>(src + L.alive)[g];
        const float reward = reinterpret_cast<const float *>(src + L.reward)[g];
        const int32_t done = reinterpret_cast<const int32_t *>(src + L.done)[g];
        const int2 mg = reinterpret_cast<const int2 *>(src + L.mag)[g];
        float coef[9];
        for (int c = 0; c < 9; c++) coef[c] = reinterpret_cast<const float *>(src + L.coefs)[g * 9 + c];
        S.hp[g] = hp;
        S.alive[g] = alive;
        S.reward[g] = reward;
        S.done[g] = done;
        reinterpret_cast<int2 *>(S.magazine)[g] = mg;
        for (int c = 0; c < 9; c++) S.rewardCoefs[g * 9 + c] = coef[c];
        if (L.lkObs >= 0) {
            const float4 *s4 = reinterpret_cast<const float4 *>(src + L.lkObs) + g * 6 * kOtherObs / 4;
            float4 *lk = reinterpret_cast<float4 *>(S.lkObs + g * 6 * kOtherObs);
            for (int q = 0; q < 6 * kOtherObs / 4; q++) lk[q] = s4[q];
            for (int q = 0; q < 18; q++) S.lkPos[g * 18 + q] = reinterpret_cast<const float *>(src + L.lkPos)[g * 18 + q];
        }
    } else if (b < G.match) {
        const int64_t w = (int64_t)(b - G.worlds) * 256 + threadIdx.x;
        if (w >= S.W) return;
        epNext[w] = reinterpret_cast<const int32_t *>(src + L.wi[kWireWI - 1])[w];
    } else {
        // [W][30] i32 episode results: 16-B pieces of the flat array (both
        // ends 256-B aligned; the last piece may be partial)
        const int64_t i = (int64_t)(b - G.match) * 256 + threadIdx.x;
        const int64_t bytes = S.W * 120;
        if (i * 16 >= bytes) return;
        if (i * 16 + 16 <= bytes) {
            reinterpret_cast<uint4 *>(S.matchResult)[i] = reinterpret_cast<const uint4 *>(src + L.match)[i];
        } else {
            for (int64_t o = i * 16; o < bytes; o += 4)
                S.matchResult[o / 4] = reinterpret_cast<const int32_t *>(src + L.match)[o / 4];
        }
    }
}

// ------------------------------------------------------------ batch copy
// gpuStreamStep's input and output copies (mgr.cpp:614-645) as one launch
// per direction (hipMemcpyAsync per tensor ran at ~1 TB/s for the 2.4 GB of
// a C3 step).  Every segment gets ceil(pieces / (256 x kCopyPieces)) blocks
// of its own (first[k] = its first block), so a block's segment is one
// wave-uniform lookup and blocks are spread over the segments by size
// (round 4 gave every segment the largest one's grid: most blocks of the
// small segments found nothing to do); each lane keeps kCopyPieces 16-B
// loads in flight before its stores, every load and store instruction
// unit-stride.  src == nullptr writes zeros (the agent maps, never written
// by the step): store-only pieces.  A segment's last piece may be partial.
constexpr int kCopyPieces = 8;
constexpr int kCopyBlockPieces = 256 * kCopyPieces;

__global__ void __launch_bounds__(256) k_copy_batch(CopyBatch b)
{
    if (b.tabDst && blockIdx.x == 0 && threadIdx.x == 0) *b.tabDst = b.tab;
    if (b.n == 0) return;
    int k = 0;
    while (k + 1 < b.n && b.first[k + 1] <= (int64_t)blockIdx.x) k++; // uniform
    const CopySeg sg = b.seg[k];
    const int64_t n16 = sg.bytes / 16;
    const int64_t p0 = ((int64_t)blockIdx.x - b.first[k]) * kCopyBlockPieces + threadIdx.x;
    const uint4 *src = static_cast<const uint4 *>(sg.src);
    uint4 *dst = static_cast<uint4 *>(sg.dst);
    if (src) {
        uint4 v[kCopyPieces];
#pragma unroll
        for (int j = 0; j < kCopyPieces; j++) {
            const int64_t p = p0 + j * 256;
            v[j] = p < n16 ? src[p] : make_uint4(0u, 0u, 0u, 0u);
        }
#pragma unroll
        for (int j = 0; j < kCopyPieces; j++) {
            const int64_t p = p0 + j * 256;
            if (p < n16) dst[p] = v[j];
        }
    } else {
#pragma unroll
        for (int j = 0; j < kCopyPieces; j++) {
            const int64_t p = p0 + j * 256;
            if (p < n16) dst[p] = make_uint4(0u, 0u, 0u, 0u);
        }
    }
    // the partial last piece (bytes % 16), by the segment's first block
    if (blockIdx.x == b.first[k] && threadIdx.x < (sg.bytes & 15)) {
        const int64_t o = n16 * 16 + threadIdx.x;
        static_cast<uint8_t *>(sg.dst)[o] = src ? static_cast<const uint8_t *>(sg.src)[o] : 0;
    }
}

static int checkW(hipError_t e) { return e == hipSuccess ? 0 : -1; }

__global__ void k_wire_err_clear(uint32_t *err) { atomicAnd(err, kWireErrDesync); }

int launchWireErrClear(uint32_t *err, void *stream)
{
    hipLaunchKernelGGL(k_wire_err_clear, dim3(1), dim3(1), 0, (hipStream_t)stream, err);
    return checkW(hipGetLastError());
}
static unsigned grid(int64_t n) { return (unsigned)((n + 255) / 256); }

int64_t wireBytes(const DevState &s, bool keyframe) { return wireLayout(s.A, s.W, keyframe).total; }

int launchWirePack(const DevState &s, char *dst, bool keyframe, uint32_t worldOffset, void *stream)
{
    hipStream_t st = (hipStream_t)stream;
    const WireLayout L = wireLayout(s.A, s.W, keyframe);
    const WirePackGrid G = wirePackGrid(s.A, s.W);
    if ((uintptr_t)s.matchResult & 15u) return -1;
    if (checkW(hipMemsetAsync(dst + offsetof(WireHeader, flags), 0, sizeof(uint32_t), st))) return -1;
    hipLaunchKernelGGL(k_wire_pack, dim3(G.total), dim3(256), 0, st, s, dst, L, G, worldOffset);
    return checkW(hipGetLastError());
}

int launchCopyBatch(const CopyBatch &bIn, void *stream)
{
    if (bIn.n <= 0 && !bIn.tabDst) return 0;
    CopyBatch b = bIn;
    b.first[0] = 0;
    for (int k = 0; k < b.n; k++)
        b.first[k + 1] = b.first[k] + std::max<int64_t>(1, (b.seg[k].bytes / 16 + kCopyBlockPieces - 1) / kCopyBlockPieces);
    const int64_t blocks = std::max<int64_t>(1, b.first[b.n]);
    hipLaunchKernelGGL(k_copy_batch, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, b);
    return checkW(hipGetLastError());
}

int launchWireUnpack(const DevState &s, const SceneDev &sc, const char *src, bool keyframe, uint32_t *err,
                     uint32_t worldOffset, const int32_t *epPrev, int32_t *epNext, void *stream)
{
    hipStream_t st = (hipStream_t)stream;
    const WireLayout L = wireLayout(s.A, s.W, keyframe);
    const WireUnpackGrid G = wireUnpackGrid(s.A, s.W);
    // the lidar quads assume 16-B aligned f32 lidar rows; the match copy
    // 16-B pieces at both ends
    if (((uintptr_t)s.fwdLidar | (uintptr_t)s.rearLidar | (uintptr_t)s.matchResult | (uintptr_t)src) & 15u) return -1;
    hipLaunchKernelGGL(k_wire_unpack, dim3(G.total), dim3(256), 0, st, s, src, L, G, err, worldOffset, epNext);
    if (checkW(hipGetLastError())) return -1;
    // the shadow seen through the message: input columns in the message,
    // outputs (and the last-known history) in the shadow; k_obs_wire skips
    // everything while the shadow is out of sync (obsGate), so a refused
    // message rebuilds nothing
    DevState v = s;
    char *m = const_cast<char *>(src);
    int k = 0;
#define MP_VIEW_F(n) v.n = reinterpret_cast<float *>(m + L.af[k++]);
    MP_WIRE_AF(MP_VIEW_F)
#undef MP_VIEW_F
    k = 0;
#define MP_VIEW_I(n) v.n = reinterpret_cast<int32_t *>(m + L.ai[k++]);
    MP_WIRE_AI(MP_VIEW_I)
#undef MP_VIEW_I
    k = 0;
#define MP_VIEW_W(n) v.n = reinterpret_cast<int32_t *>(m + L.wi[k++]);
    MP_WIRE_WI(MP_VIEW_W)
#undef MP_VIEW_W
    v.hp = reinterpret_cast<float *>(m + L.hp);
    v.alive = reinterpret_cast<float *>(m + L.alive);
    v.magazine = reinterpret_cast<int32_t *>(m + L.mag);
    v.visMask = reinterpret_cast<uint8_t *>(m + L.vis);
    v.obsGate = err;
    v.stats = nullptr;
    v.outTab = nullptr;
    WireObs wo;
    wo.packed = reinterpret_cast<const uint32_t *>(src + L.packed);
    wo.epPrev = epPrev;
    wo.keyframe = keyframe ? 1 : 0;
    return launchObservationsWire(v, sc, wo, stream);
}

} // namespace mpenv
