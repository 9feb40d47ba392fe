/*
 * oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * C interface of the CPU restatement ("oracle") of the reference's
 * world-batched Zone step.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library; the product
 * (madrona-mp-env_amd/) never links or calls it.
 */
#ifndef MPENV_ORACLE_H
#define MPENV_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_config {
    uint32_t num_worlds;
    uint32_t rand_seed;
    int32_t auto_reset;
    uint32_t sim_flags;
    uint32_t team_size;
    uint32_t world_id_offset;
    const char *scene_path;
    /* BVH built by the product's builder (same bytes the GPU traverses):
     * 64-byte nodes (mesh_bvh.hpp:61-86) and 3 float3 vertices per triangle. */
    const void *bvh_nodes;
    int32_t num_nodes;
    const float *bvh_verts;
    int32_t num_bvh_verts;
    /* Task (MPENV_TASK_*): Zone or ZoneCaptureDefend. */
    int32_t task_type;
    /* RewardMode::Flank (train_flank, mgr.cpp:1746-1750) */
    int32_t train_flank;
    /* Lidar closest-hit rule: 0 = slot order (mesh_bvh.inl:160-204 as
     * written), 1 = the round-3 octant child order, 2 = the smallest t
     * over every hit triangle -- order-independent, the
     * rule the product's k_lidar follows (DESIGN.md §2 definition 12);
     * closest hits differ only between near-coplanar overlapping triangles. */
    int32_t lidar_octant_order;
    /* pvpLidar's tree (the product's mpenv_scene_lidar_bvh, same format),
     * walked by the octant and lex rules; null = the collision tree above.
     * The slot rule (the reference's order) keeps the collision tree, the
     * reference's only tree. */
    const void *lidar_bvh_nodes;
    int32_t num_lidar_nodes;
    const float *lidar_bvh_verts;
    int32_t num_lidar_bvh_verts;
} oracle_config;

void *oracle_create(const oracle_config *cfg);
void oracle_destroy(void *h);
int oracle_export(void *h, int32_t export_id, void **ptr, int32_t *dtype,
                  int32_t *ndim, int64_t *dims);
/* Manager::init: forced reset of every world then the Init graph. */
void oracle_init(void *h);
/* One Step graph over all worlds. */
void oracle_step(void *h);
/* One Step graph over worlds [w0, w1) (caller guarantees disjoint ranges). */
void oracle_step_worlds(void *h, int32_t w0, int32_t w1);
/* Refresh MPENV_EXPORT_DEBUG_* buffers from internal state. */
void oracle_refresh_debug(void *h);
/* Record / replay / event-log modes (sim.cpp:4750-4843, 23-106): buffers
 * exported as MPENV_EXPORT_RECORD_LOG / REPLAY_LOG / EVENT_LOG /
 * PACKED_STEP_SNAPSHOT / SNAPSHOT_WRITTEN; in replay mode the caller fills
 * REPLAY_LOG before each step. */
void oracle_set_log_modes(void *h, int32_t record, int32_t replay, int32_t events);
/* Trajectory curriculum (level_gen.cpp:498-581): n CurriculumSnapshots
 * (include/mpenv.h mpenv_curriculum_snapshot), copied. */
void oracle_set_curriculum(void *h, const void *snapshots, int32_t n);
/* CPU baseline timing: runs nsteps steps over all worlds with nthreads
 * std::threads (static world partition, like ThreadPoolExecutor,
 * mgr.cpp:1863-1871).  Before each step the discrete/aim actions of step s
 * are copied from ring[(s % ring_len)] (layout [ring_len][A][6] i32:
 * 4 discrete + 2 aim).  Returns wall seconds. */
double oracle_run_threaded(void *h, int32_t nsteps, int32_t nthreads,
                           const int32_t *ring, int32_t ring_len);

/* The oracle's own navmesh (scene_path/navmesh.bin: dedup, fan
 * triangulation, adjacency) and buildAStarLookup table (mgr.cpp:946-1211),
 * built at oracle_create independently of the product's builder:
 * tris [T][3][3], adjacency [T][3], next hop [T][T]; any pointer may be null. */
int oracle_navmesh(void *h, float *tris_out, int32_t *adj_out, int32_t *astar_out, int32_t *num_tris);

/* Analysis only: out2 = {sphere casts, casts that ended at
 * t = 0} since the last reset; leaf_read_two >= 0 then resets the counters
 * and sets the sphereCastLeaf read rule (1 = two consecutive triangles, the
 * reference's; 0 = triSize triangles, for comparison). -1 only reads. */
void oracle_cast_stats(int32_t leaf_read_two, uint64_t *out2);

/* Geometry hooks for known-answer tests (mesh_bvh.inl restatement). */
int oracle_trace_ray(void *h, const float *o, const float *d, float *t_out);
float oracle_sphere_cast(void *h, const float *o, const float *d, float r,
                         float *normal_out);
/* Analysis hook (DESIGN.md §2 definition 13): ray-slab products fused (1,
 * the shared definition) or multiplied then added (0). Process-wide. */
void oracle_set_slab_fma(int32_t on);
/* n closest-hit queries (MeshBVH::traceRay): order 0 slot order, 1 octant
 * order, 2 the smallest-t rule over the BVH, 3 the same rule by brute
 * force over every triangle; o, d [n][3]; t_out, hit_out [n]. */
void oracle_trace_ray_batch(void *h, int32_t n, const float *o, const float *d, int32_t order, float *t_out,
                            int32_t *hit_out);
/* n casts of MeshBVH::sphereCast with its t_max argument (mesh_bvh.inl:743-747;
 * t_max null = FLT_MAX): o, d, n_out [n][3]; normals are (0,0,0) on a miss. */
void oracle_sphere_cast_batch(void *h, int32_t n, const float *o, const float *d, float r,
                              const float *t_max, float *t_out, float *n_out);
int oracle_trace_ray_brute(void *h, const float *o, const float *d, float *t_out);
float oracle_sphere_cast_brute(void *h, const float *o, const float *d, float r);

/* Known-answer hooks for the shared Madrona-layer definitions
 * (mpenv_core.h): fn 0 sin, 1 cos, 2 atan2(in, in2), 3 asin, 4 log,
 * 5 sqrt, 6 x / in2. */
void oracle_eval_math(int32_t fn, const float *in, const float *in2, float *out, int32_t n);
void oracle_threefry(uint32_t k0, uint32_t k1, uint32_t c0, uint32_t c1, uint32_t *out2);
void oracle_tape_actions(uint32_t seed, uint32_t step, uint32_t first_agent, int32_t n, int32_t *out6);
float oracle_capsule(const float *o, const float *d, float r, float h);

#ifdef __cplusplus
}
#endif

#endif
