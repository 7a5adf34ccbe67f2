// nascar_device.h -- per-car device code of the fused CarEnv step (gfx950).
//
// One lane owns one car.  Everything the reference does per car-step
// (src/car_env.py:_run_single_physics_step -> CarPhysics.step -> Car.update_physics
// -> b2World::Step -> LapTimer.update, then obs / reward) is restated here on
// float32 (Box2D) / float64 (Python) values with the reference's operation order,
// so results match the reference bit for bit (DESIGN.md "Parity").
//
// Box2D 2.3 (box2d-py 2.3.8, reference requirements.txt:4) is a third-party
// dependency; the subset restated is: b2World::Step/Solve/SolveTOI,
// b2ContactSolver, b2CollidePolygons, b2TimeOfImpact/b2Distance, fat-AABB proxy
// pairing and b2PolygonShape::RayCast for one dynamic box vs static boxes.
#pragma once
#include "nascar_math.h"
#include "nascar_layout.h"

#pragma clang fp contract(off)

#ifndef BLOCK
#define BLOCK 256   // threads per workgroup of the sensor kernel
#endif
#ifndef SBLOCK
#define SBLOCK 128  // threads per workgroup of the one-lane-per-car kernels (whole envs)
#endif

#ifdef NASCAR_PROFILE
// profile build only: per-wave s_memtime stamps at phase boundaries of step_kernel
__device__ unsigned long long* g_prof = nullptr;
// the launch's first workgroup in the whole grid's numbering (the sharded rollout's shards start at Params.blk0), set by
// every thread of the step and sensor kernels (PROF_B0) before their first stamp, so the shards' stamp rows do not
// collide; rows are masked into their regions, so a kernel that never sets it still writes in bounds
__shared__ int s_prof_b0;
#define PROF_B0(v) (s_prof_b0 = (v))
#define PROF_BLK ((size_t)((blockIdx.x + (unsigned)s_prof_b0) & 16383u))
#define PROF(ph) do { unsigned long long _t = __builtin_amdgcn_s_memtime(); \
    if (g_prof && (threadIdx.x & 63) == 0) g_prof[(PROF_BLK * (BLOCK / 64) + threadIdx.x / 64) * 16 + (ph)] = _t; } while (0)
#define PROFS(ph) do { unsigned long long _t = __builtin_amdgcn_s_memtime(); \
    if (g_prof && (threadIdx.x & 63) == 0) g_prof[(65536 + PROF_BLK * (BLOCK / 64) + threadIdx.x / 64) * 16 + (ph)] = _t; } while (0)
// ray_sensor_kernel stamps (any block size): rows of the sensor region by blockIdx.x * waves per block + wave
#define PROFR(ph) do { unsigned long long _t = __builtin_amdgcn_s_memtime(); \
    if (g_prof && (threadIdx.x & 63) == 0) g_prof[(65536 + PROF_BLK * (blockDim.x >> 6) + threadIdx.x / 64) * 16 + (ph)] = _t; } while (0)
// the wave's XCD (HW_REG_XCC_ID, 1-based so 0 = unstamped) into stamp slot ph of the model / sensor rows
#define PROF_XCC(ph) do { const unsigned long long _x = (__builtin_amdgcn_s_getreg((3 << 11) | 20) & 15) + 1; \
    if (g_prof && (threadIdx.x & 63) == 0) g_prof[(PROF_BLK * (BLOCK / 64) + threadIdx.x / 64) * 16 + (ph)] = _x; } while (0)
#define PROFR_XCC(ph) do { const unsigned long long _x = (__builtin_amdgcn_s_getreg((3 << 11) | 20) & 15) + 1; \
    if (g_prof && (threadIdx.x & 63) == 0) g_prof[(65536 + PROF_BLK * (blockDim.x >> 6) + threadIdx.x / 64) * 16 + (ph)] = _x; } while (0)
#define PROFR_RT(ph) do { unsigned long long _t = __builtin_amdgcn_s_memrealtime(); \
    if (g_prof && (threadIdx.x & 63) == 0) g_prof[(65536 + PROF_BLK * (blockDim.x >> 6) + threadIdx.x / 64) * 16 + (ph)] = _t; } while (0)
#define PROFS_RT(ph) do { unsigned long long _t = __builtin_amdgcn_s_memrealtime(); \
    if (g_prof && (threadIdx.x & 63) == 0) g_prof[(65536 + PROF_BLK * (BLOCK / 64) + threadIdx.x / 64) * 16 + (ph)] = _t; } while (0)
// event counters: same-address global atomics from every lane serialise (milliseconds per launch), so
// they have their own build flag and never run in a stamp (timing) build
#ifdef NASCAR_PROFILE_COUNT
#define PCOUNT(slot, v) do { if (g_prof) atomicAdd(&g_prof[2 * 65536 * 16 + (slot)], (unsigned long long)(v)); } while (0)
#else
#define PCOUNT(slot, v) do { } while (0)
#endif
#ifdef NASCAR_PROFILE_UP   // sub-phases of update_physics in slots 11-13 instead of b2_step's
#define PROFB(ph) do { } while (0)
#define PROFU(ph) PROF(ph)
#else
#define PROFB(ph) PROF(ph)
#define PROFU(ph) do { } while (0)
#endif
#define PROF_RT(slot) do { unsigned long long _t = __builtin_amdgcn_s_memrealtime(); \
    if (g_prof && (threadIdx.x & 63) == 0) g_prof[(PROF_BLK * (BLOCK / 64) + threadIdx.x / 64) * 16 + (slot)] = _t; } while (0)
// actor_kernel stamps: region after the counters, 16 slots per wave (64-thread waves, any block size)
#define APROF_BASE (2 * 65536 * 16 + 64)
#define APROF(ph) do { unsigned long long _t = __builtin_amdgcn_s_memtime(); \
    if (g_prof && (threadIdx.x & 63) == 0) g_prof[APROF_BASE + ((size_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64) * 16 + (ph)] = _t; } while (0)
#define APROF_RT(ph) do { unsigned long long _t = __builtin_amdgcn_s_memrealtime(); \
    if (g_prof && (threadIdx.x & 63) == 0) g_prof[APROF_BASE + ((size_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64) * 16 + (ph)] = _t; } while (0)
// logic_kernel stamps: region after the actor's (4096 waves x 16 slots)
#define LPROF_BASE (APROF_BASE + 4096 * 16)
#define LPROF(ph) do { unsigned long long _t = __builtin_amdgcn_s_memtime(); \
    if (g_prof && (threadIdx.x & 63) == 0) g_prof[LPROF_BASE + (PROF_BLK * (SBLOCK / 64) + threadIdx.x / 64) * 16 + (ph)] = _t; } while (0)
// per-car counters of the Box2D step (model_kernel lane of car c.pid, no atomics): region after logic's
#define CPROF_BASE (LPROF_BASE + 65536 * 16)
// per-car slots (CPROF_STRIDE per car): non-returning atomics, so a count does not wait on memory (a read-modify-
// write here put a dependent global round trip into every counted phase)
#define CPROF_STRIDE 48
#define CCOUNT(c, slot, v) do { if (g_prof) (void)atomicAdd(&g_prof[CPROF_BASE + (size_t)(c).pid * CPROF_STRIDE + (slot)], \
                                                          (unsigned long long)(v)); } while (0)
#define CTIME_BEGIN() const unsigned long long _ct0 = __builtin_amdgcn_s_memtime()
// rollout_kernel per-wave phase cycles summed over its steps: region after the per-car counters (N <= 2^20)
#define RPROF_BASE (CPROF_BASE + (size_t)(1 << 19) * CPROF_STRIDE)
#define RPROF_ADD(slot, v) do { if (g_prof && (threadIdx.x & 63) == 0) \
    g_prof[RPROF_BASE + ((size_t)blockIdx.x * (SBLOCK / 64) + threadIdx.x / 64) * 4 + (slot)] += (v); } while (0)
#define CTIME_END(c, slot) CCOUNT(c, slot, __builtin_amdgcn_s_memtime() - _ct0)
// -DNASCAR_TOI_CAPTURE (with NASCAR_PROFILE): the inputs of every computed b2TimeOfImpact job (the car's sweep as two
// float4 and the wall record), for tools/toi_bench.py; a counter word, then TCAP_MAX records of 8 words
#define TCAP_BASE (RPROF_BASE + (size_t)65536 * 5)
#define TCAP_MAX 16384
#else
#define PROF_B0(v) do { } while (0)
#define CCOUNT(c, slot, v) do { } while (0)
#define CTIME_BEGIN() do { } while (0)
#define RPROF_ADD(slot, v) do { } while (0)
#define CTIME_END(c, slot) do { } while (0)
#define PROF(ph) do { } while (0)
#define PROFS(ph) do { } while (0)
#define PROFR(ph) do { } while (0)
#define PROF_XCC(ph) do { } while (0)
#define PROFR_XCC(ph) do { } while (0)
#define PROFR_RT(ph) do { } while (0)
#define PROFS_RT(ph) do { } while (0)
#define PROFB(ph) do { } while (0)
#define PROFU(ph) do { } while (0)
#define PCOUNT(slot, v) do { } while (0)
#define PROF_RT(slot) do { } while (0)
#define APROF(ph) do { } while (0)
#define APROF_RT(ph) do { } while (0)
#define LPROF(ph) do { } while (0)
#endif

namespace nascar {

// ---------------------------------------------------------------- settings
#define B2_PI 3.14159265359f
#define LINEAR_SLOP 0.005f
#define POLY_RADIUS (2.0f * LINEAR_SLOP)
#define AABB_EXT 0.1f
#define AABB_MULT 2.0f
#define MAX_TRANSLATION 2.0f
#define MAX_ROTATION (0.5f * B2_PI)
#define BAUMGARTE 0.2f
#define TOI_BAUMGARTE 0.75f
#define MAX_LINEAR_CORRECTION 0.2f
#define VELOCITY_THRESHOLD 1.0f
#define TIME_TO_SLEEP 0.5f
#define LINEAR_SLEEP_TOL 0.01f
#define ANGULAR_SLEEP_TOL (2.0f / 180.0f * B2_PI)
#define MAX_SUBSTEPS 8
#define MAX_TOI_CONTACTS 32
#define FLT_EPS 1.1920928955078125e-07f
#define FLT_BIG 3.402823466e+38f

// car fixture (src/car.py:217-239)
#define CAR_HX ((float)(5.042 / 2.0))
#define CAR_HY ((float)(1.996 / 2.0))
#define CAR_INV_MASS (1.0f / 1500.0f)
#define CAR_I_F ((float)(1500.0 * (5.042 * 5.042 + 1.996 * 1.996) * 0.5 / 12.0))
#define CAR_INV_I (1.0f / CAR_I_F)
#define MIX_RESTITUTION 0.25f

// reference constants (src/constants/*.py), same double expressions
#define CAR_MASS 1500.0
#define GRAVITY_MS2 9.81
#define CAR_WHEELBASE 2.794
#define CAR_MAX_TORQUE 820.0
#define CAR_MAX_POWER (670.0 * 745.7)
#define CAR_MAX_SPEED_MS (200.0 * 0.44704)
#define DRAG_CONSTANT (0.5 * 1.225 * 0.38 * 2.5)
#define ROLLING_RESISTANCE_FORCE (0.015 * CAR_MASS * GRAVITY_MS2)
#define MAX_TYRE_LOAD (CAR_MASS * GRAVITY_MS2 * 2.0)
#define STATIC_LOAD_PER_TYRE (CAR_MASS * GRAVITY_MS2 / 4.0)
#define PI_D 3.141592653589793
#define RAD_PER_DEG (PI_D / 180.0)
#define DEG_PER_RAD (180.0 / PI_D)

// Load through a global-address-space pointer.  Pointers read out of memory (the track tables hang off
// Params::tracks) are generic to the compiler, which then emits flat loads; a flat load waits on both the vector
// memory and the LDS counters (and completes out of order), so every one of them serialises against the LDS
// traffic around it.  The tables are global memory, and saying so gives global_load.
// Aggregates (float4, DSeg, LWall) are copied as native 16 / 8 / 4-byte vectors: a struct copy through the
// address-space pointer would become a memcpy that forgets the address space again.
typedef unsigned int gu4 __attribute__((ext_vector_type(4)));
typedef unsigned int gu2 __attribute__((ext_vector_type(2)));
template <typename T> __device__ __forceinline__ T ldg(const T* p) {
  if constexpr (sizeof(T) % 16 == 0) {
    T r;
    const __attribute__((address_space(1))) gu4* q = (const __attribute__((address_space(1))) gu4*)p;
#pragma unroll
    for (int i = 0; i < (int)(sizeof(T) / 16); ++i) { const gu4 v = q[i]; __builtin_memcpy((char*)&r + 16 * i, &v, 16); }
    return r;
  } else if constexpr (sizeof(T) % 8 == 0) {
    T r;
    const __attribute__((address_space(1))) gu2* q = (const __attribute__((address_space(1))) gu2*)p;
#pragma unroll
    for (int i = 0; i < (int)(sizeof(T) / 8); ++i) { const gu2 v = q[i]; __builtin_memcpy((char*)&r + 8 * i, &v, 8); }
    return r;
  } else {
    return *(const __attribute__((address_space(1))) T*)p;
  }
}

// ------------------------------------------------------------------ vectors
struct V2 { float x, y; };
struct Rot { float s, c; };
struct Xf { V2 p; Rot q; };
struct Aabb { V2 lo, hi; };

__device__ __forceinline__ V2 V(float x, float y) { V2 r; r.x = x; r.y = y; return r; }
__device__ __forceinline__ V2 vadd(V2 a, V2 b) { return V(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ V2 vsub(V2 a, V2 b) { return V(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ V2 vmul(float s, V2 a) { return V(s * a.x, s * a.y); }
__device__ __forceinline__ V2 vneg(V2 a) { return V(-a.x, -a.y); }
__device__ __forceinline__ float vdot(V2 a, V2 b) { return a.x * b.x + a.y * b.y; }
__device__ __forceinline__ float vcross(V2 a, V2 b) { return a.x * b.y - a.y * b.x; }
__device__ __forceinline__ V2 vcross_vs(V2 a, float s) { return V(s * a.y, -s * a.x); }
__device__ __forceinline__ V2 vcross_sv(float s, V2 a) { return V(-s * a.y, s * a.x); }
__device__ __forceinline__ float vlen(V2 a) { return fsqrt_cr(a.x * a.x + a.y * a.y); }
__device__ __forceinline__ float vnormalize(V2* a) {
  float length = vlen(*a);
  if (length < FLT_EPS) return 0.0f;
  float inv = fdiv_cr(1.0f, length);
  a->x *= inv; a->y *= inv;
  return length;
}
__device__ __forceinline__ V2 rmul(Rot q, V2 v) { return V(q.c * v.x - q.s * v.y, q.s * v.x + q.c * v.y); }
__device__ __forceinline__ V2 rmulT(Rot q, V2 v) { return V(q.c * v.x + q.s * v.y, -q.s * v.x + q.c * v.y); }
__device__ __forceinline__ V2 xmul(Xf T, V2 v) {
  return V((T.q.c * v.x - T.q.s * v.y) + T.p.x, (T.q.s * v.x + T.q.c * v.y) + T.p.y);
}
__device__ __forceinline__ V2 xmulT(Xf T, V2 v) {
  float px = v.x - T.p.x, py = v.y - T.p.y;
  return V(T.q.c * px + T.q.s * py, -T.q.s * px + T.q.c * py);
}
__device__ __forceinline__ Xf xmulT_xx(Xf A, Xf B) {
  Xf C;
  C.q.s = A.q.c * B.q.s - A.q.s * B.q.c;
  C.q.c = A.q.c * B.q.c + A.q.s * B.q.s;
  C.p = rmulT(A.q, vsub(B.p, A.p));
  return C;
}
__device__ __forceinline__ float fminb(float a, float b) { return a < b ? a : b; }
__device__ __forceinline__ float fmaxb(float a, float b) { return a > b ? a : b; }
__device__ __forceinline__ float fclamp(float a, float lo, float hi) { return fmaxb(lo, fminb(a, hi)); }
__device__ __forceinline__ V2 vmin(V2 a, V2 b) { return V(fminb(a.x, b.x), fminb(a.y, b.y)); }
__device__ __forceinline__ V2 vmax(V2 a, V2 b) { return V(fmaxb(a.x, b.x), fmaxb(a.y, b.y)); }
__device__ __forceinline__ Rot rot_set(float a) { Rot q; glibc_sincosf(a, &q.s, &q.c); return q; }
__device__ __forceinline__ V2 zero2() { return V(0.0f, 0.0f); }

// ------------------------------------------------------------------ polygons
// b2PolygonShape::SetAsBox(hx, hy): vertices (-hx,-hy), (hx,-hy), (hx,hy), (-hx,hy) and normals (0,-1),
// (1,0), (0,1), (-1,0).  Every polygon here is such a box, so vertex / normal i is generated from i by
// sign-bit arithmetic (exact, zeros are +0 as in Box2D).  An array form sat in scratch memory under the
// lane-varying vertex indices of the contact / GJK / TOI code (hundreds of cycles per access on the
// serial chain of a touching car); an earlier select-chain form was miscompiled by hipcc -O3.
struct Poly { float hx, hy, radius; };
__device__ __forceinline__ void make_box(Poly* p, float hx, float hy) { p->hx = hx; p->hy = hy; p->radius = POLY_RADIUS; }
__device__ __forceinline__ float with_sign(float m, uint32_t neg) { return __uint_as_float(__float_as_uint(m) | (neg << 31)); }
__device__ __forceinline__ V2 pv(const Poly* p, int i) {
  const uint32_t u = (uint32_t)i;
  return V(with_sign(p->hx, (((u + 1u) >> 1) & 1u) ^ 1u), with_sign(p->hy, ((u >> 1) & 1u) ^ 1u));
}
__device__ __forceinline__ V2 pn(const Poly* p, int i) {
  const uint32_t u = (uint32_t)i, odd = u & 1u, hi = (u >> 1) & 1u;
  return V(with_sign((float)odd, hi & odd), with_sign((float)(odd ^ 1u), (hi ^ 1u) & (odd ^ 1u)));
}
__device__ __forceinline__ Aabb poly_aabb(const Poly* p, Xf xf) {
  V2 lower = xmul(xf, pv(p, 0)), upper = lower;
#pragma unroll
  for (int i = 1; i < 4; ++i) { V2 v = xmul(xf, pv(p, i)); lower = vmin(lower, v); upper = vmax(upper, v); }
  V2 r = V(p->radius, p->radius);
  Aabb a; a.lo = vsub(lower, r); a.hi = vadd(upper, r);
  return a;
}
__device__ __forceinline__ bool overlap(Aabb a, Aabb b) {
  V2 d1 = vsub(b.lo, a.hi), d2 = vsub(a.lo, b.hi);
  if (d1.x > 0.0f || d1.y > 0.0f) return false;
  if (d2.x > 0.0f || d2.y > 0.0f) return false;
  return true;
}
__device__ __forceinline__ bool contains(Aabb a, Aabb b) {
  bool r = true;
  r = r && a.lo.x <= b.lo.x; r = r && a.lo.y <= b.lo.y;
  r = r && b.hi.x <= a.hi.x; r = r && b.hi.y <= a.hi.y;
  return r;
}

// wall table (built on the host from the reference wall builder): 32 bytes per wall, so model_kernel can stage a
// whole track's table in LDS next to its TOI work lists at its occupancy; the broadphase fat AABBs are a separate
// float4 array (WallSet::fat: read by the contact-list culls only)
struct LWall {
  float px, py, qs, qc;   // b2Body transform
  float hx, hy, ang;      // half extents, angle
  int key;                // listener key id (src/car_physics.py:747)
};
__device__ __forceinline__ Xf wall_xf(const LWall& w) { Xf t; t.p = V(w.px, w.py); t.q.s = w.qs; t.q.c = w.qc; return t; }
__device__ __forceinline__ Aabb fat_box(float4 f) { Aabb a; a.lo = V(f.x, f.y); a.hi = V(f.z, f.w); return a; }

// Uniform grid of wall lists over a track (built on the host, nascar_add_track).
// Cell (ix, iy) covers [ox + ix*cell, ox + (ix+1)*cell) x [...]; its list holds every
// wall that can matter to a query centred in the cell:
//   bp: walls whose fat AABB overlaps the cell grown by `reach` (query half-extent
//       <= reach - 0.05, else the caller scans all walls); ascending wall index, so the
//       broadphase pair order (b2BroadPhase::UpdatePairs sorts pairs) is unchanged.
//   sn: walls whose culling circle comes within 250 m of the cell (distance sensors),
//       nearest first.
struct WallGrid {
  float ox, oy, inv_cell, reach;
  int nx, ny;
  const int* start;        // [nx*ny + 1]
  const uint16_t* idx;
  const float4* box;       // bp only: fat AABB (lo.x, lo.y, hi.x, hi.y) of wall idx[k], padded by BP_BATCH entries
};
#ifndef BP_BATCH
#define BP_BATCH 4   // broadphase candidates whose boxes are loaded together (0: one wall record at a time)
#endif
struct WallSet {
  const LWall* W; int nw;
  WallGrid bp, sn;
  const float4* fat;      // [nw] broadphase fat AABB (lo.x, lo.y, hi.x, hi.y)
  DContact* ct_all = nullptr;   // the global contact records ([N][MAXC]) when a car's may be held in LDS (model_kernel)
};

// list of the cell containing (x, y), or false when outside the grid
__device__ __forceinline__ bool grid_list(const WallGrid& g, float x, float y, int& beg, int& end) {
  if (!g.start) return false;
  const float fx = (x - g.ox) * g.inv_cell, fy = (y - g.oy) * g.inv_cell;
  if (!(fx >= 0.0f && fy >= 0.0f && fx < (float)g.nx && fy < (float)g.ny)) return false;
  const int cell = (int)fy * g.nx + (int)fx;
  beg = ldg(g.start + cell); end = ldg(g.start + cell + 1);
  return true;
}

// ------------------------------------------------------------------ per-car register state
struct Car {
  // b2Body
  V2 c; float a; V2 v; float w; Xf xf; float sleep; int awake;
  V2 force; float torque; V2 c0; float a0; float alpha0;
  Aabb fat; int moved; float invdt0;
  int nct, overflow;
  int pid;            // car index (its global contact records when they are moved out of LDS; profile counters)
  // Car / TyreManager (float64 like the reference's Python)
  double thr_in, brk_in, str_in, thr, brk, steer;
  double rpm, pvx, pvy, lfm, slip, bank;
  double load[4], temp[4], wear[4], fric[4];
  int acc_len, acc_head;
  // CarCollisionListener
  int imp_present, nact; double imp;
  // LapTimer
  int lt_timing, lt_has_last, lt_has_best, lt_crossed, lt_has_pos, lt_laps;
  double lt_start, lt_cur, lt_last, lt_best, lt_px, lt_py, lt_dist;
  // CarEnv bookkeeping
  int disabled, just_disabled, has_stuck_start, first_step, prev_laps;
  double cum_impact, stuck_dur, stuck_sx, stuck_sy, prev_px, prev_py, prog_hist, back, prev_back, imp_at_obs;
  float cum_reward, cum_reward_info;
  // per-car global views (AoS lists)
  DContact* ct;       // [MAXC] (global, or model_kernel's LDS slots)
  int ct_hw;          // LDS slots: records written this step (live or dead), all copied back to the global ones
  int* act_key;       // [MAXC]
  float* act_n;       // [MAXC][2]
  double* acc;        // [20] ring (long, lat)
};

// A car's contact records may live in LDS for the Box2D step (model_kernel, CT_LDS_CAP records per lane): every
// b2Contact access is then an LDS round trip instead of a global one.  A car whose list grows past the LDS slots
// moves its records back to its global ones first (same records, same order), and model_car writes LDS records
// back after the step.
#ifndef CT_LDS_CAP
#define CT_LDS_CAP 4   // 2 / 3 / 4 / 5 / 6 slots: 161 / 156 / 153 / 154 / 155 us/step sharded (5+: 2 workgroups per CU)
#endif
__device__ __forceinline__ bool ct_in_lds(const Car& c) {
  return __builtin_amdgcn_is_shared((const __attribute__((address_space(0))) void*)c.ct);
}
// before a contact is prepended: room for one more record where the list lives
// (the dead records past nct are copied too, so the global image is the one the all-global path leaves)
__device__ __forceinline__ void ct_make_room(Car& c, const WallSet& S) {
  if (S.ct_all && ct_in_lds(c)) {
    if (c.nct >= CT_LDS_CAP) {
      DContact* g = S.ct_all + (size_t)c.pid * MAXC;
      const int nrec = max(c.nct, c.ct_hw);   // live records and the dead ones earlier removals left behind
      for (int i = 0; i < nrec; ++i) g[i] = c.ct[i];
      c.ct = g;
    } else {
      c.ct_hw = max(c.ct_hw, c.nct + 1);
    }
  }
}

// ------------------------------------------------------------------ listener (src/car_physics.py:693-864)
__device__ inline void lis_begin(Car& c, int key, V2 n) {
  int found = -1;
  for (int i = 0; i < c.nact; ++i) if (c.act_key[i] == key) { found = i; break; }
  if (found >= 0) { c.act_n[found * 2] = n.x; c.act_n[found * 2 + 1] = n.y; }
  else if (c.nact < MAXC) { c.act_key[c.nact] = key; c.act_n[c.nact * 2] = n.x; c.act_n[c.nact * 2 + 1] = n.y; c.nact++; }
  if (!c.imp_present) { c.imp_present = 1; c.imp = 0.0; }
}
__device__ inline void lis_end(Car& c, int key) {
  for (int i = 0; i < c.nact; ++i) if (c.act_key[i] == key) {
    for (int j = i; j < c.nact - 1; ++j) { c.act_key[j] = c.act_key[j + 1]; c.act_n[j * 2] = c.act_n[j * 2 + 2]; c.act_n[j * 2 + 1] = c.act_n[j * 2 + 3]; }
    c.nact--; break;
  }
  if (c.nact == 0) { c.imp_present = 1; c.imp = 0.0; }
}
__device__ inline void lis_post(Car& c, int count, float n0, float n1) {
  if (count <= 0) return;
  double total = 0.0;
  total += (double)n0;
  if (count > 1) total += (double)n1;
  if (c.imp_present) c.imp = pymax(c.imp, total);
}

// ------------------------------------------------------------------ body helpers
__device__ __forceinline__ void set_awake(Car& c) { if (!c.awake) { c.awake = 1; c.sleep = 0.0f; } }
__device__ __forceinline__ void sync_transform(Car& c) { c.xf.q = rot_set(c.a); c.xf.p = vsub(c.c, rmul(c.xf.q, zero2())); }
__device__ __forceinline__ void apply_force(Car& c, V2 f, V2 point) {
  set_awake(c); c.force = vadd(c.force, f); c.torque += vcross(vsub(point, c.c), f);
}
__device__ __forceinline__ void apply_force_center(Car& c, V2 f) { set_awake(c); c.force = vadd(c.force, f); }
__device__ __forceinline__ void apply_torque(Car& c, float t) { set_awake(c); c.torque += t; }

__device__ __forceinline__ void move_proxy(Car& c, Xf xf1, Xf xf2) {
  Poly cp; make_box(&cp, CAR_HX, CAR_HY);
  Aabb a1 = poly_aabb(&cp, xf1), a2 = poly_aabb(&cp, xf2), aabb;
  aabb.lo = vmin(a1.lo, a2.lo); aabb.hi = vmax(a1.hi, a2.hi);
  V2 disp = vsub(xf2.p, xf1.p);
  if (contains(c.fat, aabb)) return;
  Aabb b = aabb; V2 r = V(AABB_EXT, AABB_EXT);
  b.lo = vsub(b.lo, r); b.hi = vadd(b.hi, r);
  V2 d = vmul(AABB_MULT, disp);
  if (d.x < 0.0f) b.lo.x += d.x; else b.hi.x += d.x;
  if (d.y < 0.0f) b.lo.y += d.y; else b.hi.y += d.y;
  c.fat = b; c.moved = 1;
}
__device__ __forceinline__ void sync_fixtures(Car& c) {
  Xf xf1; xf1.q = rot_set(c.a0); xf1.p = vsub(c.c0, rmul(xf1.q, zero2()));
  move_proxy(c, xf1, c.xf);
}

// b2ContactManager::AddPair for wall j whose fat AABB overlaps the car's (new contacts are prepended)
__device__ inline void add_pair(Car& c, const WallSet& S, int j) {
    bool exists = false;
    for (int i = 0; i < c.nct; ++i) if (c.ct[i].wall == j) { exists = true; break; }
    if (exists) return;
    if (c.nct >= MAXC) { c.overflow = 1; return; }
    ct_make_room(c, S);
    for (int i = c.nct; i > 0; --i) c.ct[i] = c.ct[i - 1];
    DContact z;
    z.wall = j; z.flags = CT_ENABLED; z.mtype = 0; z.pointCount = 0;
    z.lnx = z.lny = z.lpx = z.lpy = 0.0f;
    for (int q = 0; q < 2; ++q) { z.pt[q].lx = z.pt[q].ly = z.pt[q].ni = z.pt[q].ti = 0.0f; z.pt[q].id = 0u; }
    z.toi = 1.0f; z.toiCount = 0;
    c.ct[0] = z;
    c.nct++;
    set_awake(c);
}
// b2BroadPhase::UpdatePairs + b2ContactManager::AddPair (ascending wall proxy id, prepend)
__device__ inline void find_new_contacts(Car& c, const WallSet& S) {
#ifdef NASCAR_KO_FIND
  c.moved = 0; return;
#endif
  if (!c.moved) return;
  c.moved = 0;
  const LWall* W = S.W;
  int beg = 0, end = S.nw;
  const uint16_t* list = nullptr;
  {
    const float hx = 0.5f * (c.fat.hi.x - c.fat.lo.x), hy = 0.5f * (c.fat.hi.y - c.fat.lo.y);
    const float cx = 0.5f * (c.fat.hi.x + c.fat.lo.x), cy = 0.5f * (c.fat.hi.y + c.fat.lo.y);
    if (hx <= S.bp.reach - 0.05f && hy <= S.bp.reach - 0.05f && grid_list(S.bp, cx, cy, beg, end)) list = S.bp.idx;
    else { beg = 0; end = S.nw; CCOUNT(c, 8, 1); }
  }
#if BP_BATCH > 0
  if (list && S.bp.box) {
    // the cell's candidate boxes stored in list order: BP_BATCH independent loads per round instead of a
    // dependent (index -> wall record) pair per candidate; same candidates, same ascending order
    const float4* __restrict__ box = S.bp.box;
    for (int k = beg; k < end; k += BP_BATCH) {
      float4 b[BP_BATCH];
#pragma unroll
      for (int u = 0; u < BP_BATCH; ++u) b[u] = ldg(box + k + u);   // in bounds: the array is padded by BP_BATCH
#pragma unroll
      for (int u = 0; u < BP_BATCH; ++u) {
        if (k + u >= end) break;
        Aabb a; a.lo = V(b[u].x, b[u].y); a.hi = V(b[u].z, b[u].w);
        if (overlap(c.fat, a)) add_pair(c, S, (int)ldg(list + k + u));
      }
    }
    return;
  }
#endif
  for (int k = beg; k < end; ++k) {
    const int j = list ? (int)ldg(list + k) : k;
    if (!overlap(c.fat, fat_box(ldg(S.fat + j)))) continue;
    bool exists = false;
    for (int i = 0; i < c.nct; ++i) if (c.ct[i].wall == j) { exists = true; break; }
    if (exists) continue;
    if (c.nct >= MAXC) { c.overflow = 1; continue; }
    ct_make_room(c, S);
    for (int i = c.nct; i > 0; --i) c.ct[i] = c.ct[i - 1];
    DContact z;
    z.wall = j; z.flags = CT_ENABLED; z.mtype = 0; z.pointCount = 0;
    z.lnx = z.lny = z.lpx = z.lpy = 0.0f;
    for (int q = 0; q < 2; ++q) { z.pt[q].lx = z.pt[q].ly = z.pt[q].ni = z.pt[q].ti = 0.0f; z.pt[q].id = 0u; }
    z.toi = 1.0f; z.toiCount = 0;
    c.ct[0] = z;
    c.nct++;
    set_awake(c);
  }
}
__device__ inline void remove_contact(Car& c, int i) {
  for (int j = i; j < c.nct - 1; ++j) c.ct[j] = c.ct[j + 1];
  c.nct--;
}

// ------------------------------------------------------------------ b2CollidePolygons
struct Clip { V2 v; uint32_t id; };
__device__ __forceinline__ uint32_t cf_key(int ia, int ib, int ta, int tb) {
  return (uint32_t)(ia & 255) | ((uint32_t)(ib & 255) << 8) | ((uint32_t)(ta & 255) << 16) | ((uint32_t)(tb & 255) << 24);
}
__device__ inline float find_max_separation(int* edgeIndex, const Poly* p1, Xf xf1, const Poly* p2, Xf xf2) {
  Xf xf = xmulT_xx(xf2, xf1);
  int best = 0; float maxSep = -FLT_BIG;
  for (int i = 0; i < 4; ++i) {
    V2 n = rmul(xf.q, pn(p1, i));
    V2 v1 = xmul(xf, pv(p1, i));
    float si = FLT_BIG;
    for (int j = 0; j < 4; ++j) { float sij = vdot(n, vsub(pv(p2, j), v1)); if (sij < si) si = sij; }
    if (si > maxSep) { maxSep = si; best = i; }
  }
  *edgeIndex = best;
  return maxSep;
}
__device__ inline void find_incident_edge(Clip& c0, Clip& c1, const Poly* p1, Xf xf1, int edge1, const Poly* p2, Xf xf2) {
  V2 normal1 = rmulT(xf2.q, rmul(xf1.q, pn(p1, edge1)));
  int index = 0; float minDot = FLT_BIG;
  for (int i = 0; i < 4; ++i) { float d = vdot(normal1, pn(p2, i)); if (d < minDot) { minDot = d; index = i; } }
  int i1 = index, i2 = i1 + 1 < 4 ? i1 + 1 : 0;
  c0.v = xmul(xf2, pv(p2, i1)); c0.id = cf_key(edge1, i1, 1, 0);
  c1.v = xmul(xf2, pv(p2, i2)); c1.id = cf_key(edge1, i2, 1, 0);
}
// b2ClipSegmentToLine with the two outputs as named values (no dynamically indexed array)
__device__ inline int clip_segment(Clip& o0, Clip& o1, const Clip& i0, const Clip& i1, V2 normal, float offset, int vertexIndexA) {
  int numOut = 0;
  float d0 = vdot(normal, i0.v) - offset;
  float d1 = vdot(normal, i1.v) - offset;
  if (d0 <= 0.0f) { o0 = i0; numOut = 1; }
  if (d1 <= 0.0f) { if (numOut == 0) o0 = i1; else o1 = i1; ++numOut; }
  if (d0 * d1 < 0.0f) {   // d0, d1 of opposite signs: exactly one was kept, the new point is the second
    float interp = fdiv_cr(d0, d0 - d1);
    Clip cv;
    cv.v = vadd(i0.v, vmul(interp, vsub(i1.v, i0.v)));
    cv.id = cf_key(vertexIndexA, (int)((i0.id >> 8) & 255), 0, 1);
    if (numOut == 0) o0 = cv; else o1 = cv;
    ++numOut;
  }
  return numOut;
}
// writes manifold into ct (type, localNormal, localPoint, pointCount, points' localPoint/id; impulses zeroed)
__device__ inline void collide_polygons(DContact& m, const Poly* pA, Xf xfA, const Poly* pB, Xf xfB) {
  m.pointCount = 0;
  float totalRadius = pA->radius + pB->radius;
  int edgeA = 0; float sepA = find_max_separation(&edgeA, pA, xfA, pB, xfB);
  if (sepA > totalRadius) return;
  int edgeB = 0; float sepB = find_max_separation(&edgeB, pB, xfB, pA, xfA);
  if (sepB > totalRadius) return;
  const Poly *poly1, *poly2; Xf xf1, xf2; int edge1; int flip;
  const float k_tol = 0.1f * LINEAR_SLOP;
  if (sepB > sepA + k_tol) { poly1 = pB; poly2 = pA; xf1 = xfB; xf2 = xfA; edge1 = edgeB; m.mtype = 2; flip = 1; }
  else { poly1 = pA; poly2 = pB; xf1 = xfA; xf2 = xfB; edge1 = edgeA; m.mtype = 1; flip = 0; }
  Clip inc0, inc1;
  find_incident_edge(inc0, inc1, poly1, xf1, edge1, poly2, xf2);
  int iv1 = edge1, iv2 = edge1 + 1 < 4 ? edge1 + 1 : 0;
  V2 v11 = pv(poly1, iv1), v12 = pv(poly1, iv2);
  V2 localTangent = vsub(v12, v11);
  vnormalize(&localTangent);
  V2 localNormal = vcross_vs(localTangent, 1.0f);
  V2 planePoint = vmul(0.5f, vadd(v11, v12));
  V2 tangent = rmul(xf1.q, localTangent);
  V2 normal = vcross_vs(tangent, 1.0f);
  v11 = xmul(xf1, v11); v12 = xmul(xf1, v12);
  float frontOffset = vdot(normal, v11);
  float sideOffset1 = -vdot(tangent, v11) + totalRadius;
  float sideOffset2 = vdot(tangent, v12) + totalRadius;
  Clip a0, a1, b0, b1;
  int np = clip_segment(a0, a1, inc0, inc1, vneg(tangent), sideOffset1, iv1);
  if (np < 2) return;
  np = clip_segment(b0, b1, a0, a1, tangent, sideOffset2, iv2);
  if (np < 2) return;
  m.lnx = localNormal.x; m.lny = localNormal.y; m.lpx = planePoint.x; m.lpy = planePoint.y;
  int pc = 0;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const Clip& cq = i == 0 ? b0 : b1;
    float separation = vdot(normal, cq.v) - frontOffset;
    if (separation <= totalRadius) {
      V2 lp = xmulT(xf2, cq.v);
      uint32_t id = cq.id;
      if (flip) {
        uint32_t ia = id & 255, ib = (id >> 8) & 255, ta = (id >> 16) & 255, tb = (id >> 24) & 255;
        id = cf_key((int)ib, (int)ia, (int)tb, (int)ta);
      }
      DPoint q; q.lx = lp.x; q.ly = lp.y; q.id = id; q.ni = 0.0f; q.ti = 0.0f;
      if (pc == 0) m.pt[0] = q; else m.pt[1] = q;
      ++pc;
    }
  }
  m.pointCount = pc;
}

// b2WorldManifold::Initialize
__device__ inline void world_manifold(const DContact& m, Xf xfA, Xf xfB, V2* normal, V2 pts[2]) {
  const float rA = POLY_RADIUS, rB = POLY_RADIUS;
  if (m.pointCount == 0) return;
  V2 ln = V(m.lnx, m.lny), lp = V(m.lpx, m.lpy);
  if (m.mtype == 1) {
    V2 n = rmul(xfA.q, ln), planePoint = xmul(xfA, lp);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if (i >= m.pointCount) break;
      V2 clipPoint = xmul(xfB, V(m.pt[i].lx, m.pt[i].ly));
      V2 cA = vadd(clipPoint, vmul(rA - vdot(vsub(clipPoint, planePoint), n), n));
      V2 cB = vsub(clipPoint, vmul(rB, n));
      pts[i] = vmul(0.5f, vadd(cA, cB));
    }
    *normal = n;
  } else {
    V2 n = rmul(xfB.q, ln), planePoint = xmul(xfB, lp);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if (i >= m.pointCount) break;
      V2 clipPoint = xmul(xfA, V(m.pt[i].lx, m.pt[i].ly));
      V2 cB = vadd(clipPoint, vmul(rB - vdot(vsub(clipPoint, planePoint), n), n));
      V2 cA = vsub(clipPoint, vmul(rA, n));
      pts[i] = vmul(0.5f, vadd(cA, cB));
    }
    *normal = vneg(n);
  }
}

// b2Contact::Update
__device__ inline void contact_update(Car& c, int ci, const LWall* W) {
  PCOUNT(14, 1); CCOUNT(c, 5, 1);
  DContact ct = c.ct[ci];   // register copy (one burst of loads), written back once below
  const DContact old = ct;
  ct.flags |= CT_ENABLED;
  bool was = (ct.flags & CT_TOUCH) != 0;
  Poly pa, pb; make_box(&pa, CAR_HX, CAR_HY);
  const LWall wl = ldg(W + ct.wall);   // the wall table is global (ldg: global, not flat, loads)
  make_box(&pb, wl.hx, wl.hy);
  Xf xfB = wall_xf(wl);
  collide_polygons(ct, &pa, c.xf, &pb, xfB);
  bool touching = ct.pointCount > 0;
#pragma unroll
  for (int i = 0; i < 2; ++i) {   // warm-start impulses of the old point with the same feature id (first match)
    if (i >= ct.pointCount) break;
    ct.pt[i].ni = 0.0f; ct.pt[i].ti = 0.0f;
    if (old.pointCount > 0 && old.pt[0].id == ct.pt[i].id) { ct.pt[i].ni = old.pt[0].ni; ct.pt[i].ti = old.pt[0].ti; }
    else if (old.pointCount > 1 && old.pt[1].id == ct.pt[i].id) { ct.pt[i].ni = old.pt[1].ni; ct.pt[i].ti = old.pt[1].ti; }
  }
  if (touching != was) set_awake(c);
  if (touching) ct.flags |= CT_TOUCH; else ct.flags &= ~CT_TOUCH;
  c.ct[ci] = ct;
  if (!was && touching) {
    V2 n = zero2(), pts[2];
    world_manifold(ct, c.xf, xfB, &n, pts);
    lis_begin(c, wl.key, n);
  }
  if (was && !touching) lis_end(c, wl.key);
}

// b2Contact::Update split in two for SolveTOI's events (wave-cooperative manifolds, see solve_toi): the manifold
// b2CollidePolygons computes from the car's transform and the wall (any lane), and the rest of Update on the owner's
// record.  collide_polygons leaves a record's fields untouched past an early exit, so the packed result says which
// fields it wrote (stage 0: pointCount only, 1: + type, 2: + local normal / point and the first pc points).
struct ManiRes { float4 a, b, c; };
#define MANI_UNSET 0x7fc0deadu   // a NaN collide_polygons never writes to localNormal.x (sentinel: stage 2 not reached)
__device__ inline ManiRes contact_manifold(Xf xfA, const LWall& wl) {
  Poly pa, pb; make_box(&pa, CAR_HX, CAR_HY); make_box(&pb, wl.hx, wl.hy);
  DContact m;
  m.mtype = -1; m.lnx = __uint_as_float(MANI_UNSET); m.pointCount = 0;
  m.lny = m.lpx = m.lpy = 0.0f;
  for (int q = 0; q < 2; ++q) { m.pt[q].lx = m.pt[q].ly = 0.0f; m.pt[q].id = 0u; }
  collide_polygons(m, &pa, xfA, &pb, wall_xf(wl));
  const int stage = __float_as_uint(m.lnx) != MANI_UNSET ? 2 : (m.mtype >= 0 ? 1 : 0);
  ManiRes r;
  r.a = make_float4(__int_as_float(stage | (m.pointCount << 2) | ((m.mtype & 3) << 4)), m.lnx, m.lny, m.lpx);
  r.b = make_float4(m.lpy, m.pt[0].lx, m.pt[0].ly, __uint_as_float(m.pt[0].id));
  r.c = make_float4(m.pt[1].lx, m.pt[1].ly, __uint_as_float(m.pt[1].id), 0.0f);
  return r;
}
// b2Contact::Update of contact ci with its manifold from contact_manifold (the same steps as contact_update)
__device__ inline void contact_apply(Car& c, int ci, const LWall* W, const ManiRes& r) {
  PCOUNT(14, 1); CCOUNT(c, 5, 1);
  DContact ct = c.ct[ci];
  const DContact old = ct;
  ct.flags |= CT_ENABLED;
  bool was = (ct.flags & CT_TOUCH) != 0;
  const int h = __float_as_int(r.a.x), stage = h & 3, pc = (h >> 2) & 3;
  ct.pointCount = 0;
  if (stage >= 1) ct.mtype = (h >> 4) & 3;
  if (stage == 2) {
    ct.lnx = r.a.y; ct.lny = r.a.z; ct.lpx = r.a.w; ct.lpy = r.b.x;
    if (pc > 0) { ct.pt[0].lx = r.b.y; ct.pt[0].ly = r.b.z; ct.pt[0].id = __float_as_uint(r.b.w); ct.pt[0].ni = 0.0f; ct.pt[0].ti = 0.0f; }
    if (pc > 1) { ct.pt[1].lx = r.c.x; ct.pt[1].ly = r.c.y; ct.pt[1].id = __float_as_uint(r.c.z); ct.pt[1].ni = 0.0f; ct.pt[1].ti = 0.0f; }
    ct.pointCount = pc;
  }
  bool touching = ct.pointCount > 0;
#pragma unroll
  for (int i = 0; i < 2; ++i) {   // warm-start impulses of the old point with the same feature id (first match)
    if (i >= ct.pointCount) break;
    ct.pt[i].ni = 0.0f; ct.pt[i].ti = 0.0f;
    if (old.pointCount > 0 && old.pt[0].id == ct.pt[i].id) { ct.pt[i].ni = old.pt[0].ni; ct.pt[i].ti = old.pt[0].ti; }
    else if (old.pointCount > 1 && old.pt[1].id == ct.pt[i].id) { ct.pt[i].ni = old.pt[1].ni; ct.pt[i].ti = old.pt[1].ti; }
  }
  if (touching != was) set_awake(c);
  if (touching) ct.flags |= CT_TOUCH; else ct.flags &= ~CT_TOUCH;
  c.ct[ci] = ct;
  if (!was && touching) {
    const LWall wl = ldg(W + ct.wall);
    V2 n = zero2(), pts[2];
    world_manifold(ct, c.xf, wall_xf(wl), &n, pts);
    lis_begin(c, wl.key, n);
  }
  if (was && !touching) lis_end(c, ldg(&W[ct.wall].key));
}

// b2ContactManager::Collide
// ------------------------------------------------------------------ wave-cooperative work lists (LDS, per wave)
// Per-car Box2D work whose size varies by car (a car's TOI pairs) is listed per lane and computed by every
// present lane of the wave, so a wave's time follows its total work rather than its busiest car.  (The same
// scheme for b2World::Collide's manifolds was parity-green but measured neutral: 118.5 vs 118.8 us.)
#define TOI_JOBCAP 64     // b2TimeOfImpact pairs per compute round per wave (more pairs: further rounds)
struct ToiWaveLDS { float4 sw0[64], sw1[64]; int2 job[TOI_JOBCAP]; float res[TOI_JOBCAP]; };
#define MANI_JOBCAP 32    // event manifolds per wave and scan computed cooperatively (the rest by their owners)
struct ManiWaveLDS { float4 xf[64]; int2 job[MANI_JOBCAP]; ManiRes res[MANI_JOBCAP]; };
#define BP_JOBCAP 128     // broadphase candidate tests per wave and round
struct BpWaveLDS { float4 fat[64]; int2 job[BP_JOBCAP]; unsigned int hit[64][2]; };
// b2ContactSolver constraint of one (car, wall) contact (register-resident for small islands; see solve_island)
struct VCP { V2 rA, rB; float ni, ti, nm, tm, vb; };
struct VC {
  VCP p[2]; V2 normal; float nm[4]; float K[4]; int pointCount;
  V2 cB; float aB; V2 vB; float wB;
  V2 ln, lp, lps[2]; int pcount, type, ci;
  Rot qB; uint32_t aB0;   // the static wall's b2Rot (its body transform) and the angle bits it was set from
};
// the general (more than ISLAND_MID contacts) island's constraints, one lane at a time (solve_island_general)
struct IslandWaveLDS { VC vc[MAX_ISLAND]; };
union WaveLDS { ToiWaveLDS toi; ManiWaveLDS mani; BpWaveLDS bp; IslandWaveLDS island; };
static_assert(sizeof(IslandWaveLDS) <= sizeof(ToiWaveLDS), "the island area must not grow the wave's LDS work area");
__shared__ WaveLDS g_wave_lds[SBLOCK / 64];   // model_kernel / rollout_kernel (the Box2D step)
__device__ __forceinline__ void wave_lds_sync() {   // a wave's LDS writes visible to its later LDS reads
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ int popc64(unsigned long long x) { return __popcll(x); }
// lanes below this one in mask m
__device__ __forceinline__ int rank_in(unsigned long long m) {
  const unsigned long long below = __lane_id() == 0 ? 0ull : (~0ull >> (64 - __lane_id()));
  return popc64(m & below);
}

__device__ inline void collide(Car& c, const WallSet& S) {
  const LWall* W = S.W;
  int i = 0;
  while (i < c.nct) {
    if (!c.awake) { ++i; continue; }
    const int wall = c.ct[i].wall;
    if (!overlap(c.fat, fat_box(ldg(S.fat + wall)))) {
      bool touching = (c.ct[i].flags & CT_TOUCH) != 0;
      remove_contact(c, i);
      if (touching) lis_end(c, ldg(&W[wall].key));
      continue;
    }
    contact_update(c, i, W);
    ++i;
  }
}

// ------------------------------------------------------------------ b2ContactSolver
// b2Rot::Set(aB) of the static body B inside the solvers: B never moves (mB = iB = 0), so aB keeps the wall's angle
// bit for bit and its rotation is the wall's body transform (glibc sinf/cosf of that same float, computed when the
// wall was created) -- no sincosf per solver point.  Any other angle (only possible through non-finite impulses)
// takes the full b2Rot::Set.
__device__ __forceinline__ Rot rot_static(float a, uint32_t a0bits, Rot q0) {
  return __float_as_uint(a) == a0bits ? q0 : rot_set(a);
}
struct BodyState { V2 c; float a; V2 v; float w; };
// unroll count of the per-contact loops below: full for islands of <= 2 contacts (register-resident), else a loop
#define UNROLL_SMALL NUNR<NMAX>::v
// A contact constraint of the general (scratch-memory) island is copied into registers for its loop body and
// written back at its end: one burst of independent scratch loads per contact and pass instead of a dependent
// scratch round trip per field use (register-resident small islands: the same code, the copies fold away)
#ifndef ISLAND_COPY
#define ISLAND_COPY 0   // measured: 81 VGPRs spilled kernel-wide, 212 vs 160 us/step (off)
#endif
#if ISLAND_COPY
#define VC_BEGIN(i) VC v = vc[i]
#define VC_END(i) vc[i] = v
#else
#define VC_BEGIN(i) VC& v = vc[i]
#define VC_END(i) (void)0
#endif
#ifndef ISLAND_MID
// islands of 3 .. ISLAND_MID contacts also solved register-resident (0: off).  2 (round 4): 3-contact islands go to the
// LDS general solver -- the fully unrolled 3-contact register solver took ~50 k cycles against ~19 k for 1-2 contacts,
// and dropping it leaves model_kernel / model_logic_kernel spill-free (233 / 244 VGPRs instead of 256 with 15 / 22
// spilled): driver's command 148.1 / 149.7 -> 143.3 / 144.8 us per step.  (3 measured faster in round 2, before the
// general island moved out of scratch memory; 4 slower.)
#define ISLAND_MID 2
#endif
// ISLAND_TWO = 2: islands of 1-2 contacts have their own register-resident solver; 0: they share the
// ISLAND_MID one (one solver instance less per island kind: a wave whose lanes hold islands of 1 and of 3 contacts
// then runs one solver, not two in turn)
#ifndef ISLAND_TWO
#define ISLAND_TWO 2
#endif
template <int NMAX> struct NUNR { static constexpr int v = NMAX <= 2 || NMAX == ISLAND_MID ? NMAX : 1; };
// The solvers' iteration loops (6 velocity, 4 / 20 position iterations) index nothing per iteration, so rolled
// loops keep the constraints in the same registers; unrolled, each island size's solver was copied six times over
// (cs_solve_velocity alone was 34 KB of model_kernel's 295 KB of code, a kernel far beyond the instruction cache).
#ifndef SOLVER_ITER_UNROLL
#define SOLVER_ITER_UNROLL 0
#endif
#if SOLVER_ITER_UNROLL
#define SOLVER_ITER_LOOP
#else
#define SOLVER_ITER_LOOP _Pragma("unroll 1")
#endif

template <int NMAX> __device__ __forceinline__ void cs_init(VC* vc, int n, const Car& c, const int* cidx, const LWall* W, bool warm, float dtRatio) {
#pragma unroll UNROLL_SMALL   // registers for small islands; the general bound stays a loop
  for (int i = 0; i < NMAX; ++i) {
    if (i >= n) break;
    const DContact& ct = c.ct[cidx[i]];
    VC_BEGIN(i);
    v.ci = cidx[i];
    v.pointCount = ct.pointCount;
    const LWall wl = ldg(W + ct.wall);
    v.cB = V(wl.px, wl.py); v.aB = wl.ang; v.vB = zero2(); v.wB = 0.0f;
    v.qB.s = wl.qs; v.qB.c = wl.qc; v.aB0 = __float_as_uint(wl.ang);
    v.ln = V(ct.lnx, ct.lny); v.lp = V(ct.lpx, ct.lpy); v.pcount = ct.pointCount; v.type = ct.mtype;
    v.K[0] = v.K[1] = v.K[2] = v.K[3] = 0.0f; v.nm[0] = v.nm[1] = v.nm[2] = v.nm[3] = 0.0f;
    for (int j = 0; j < 2; ++j) {
      v.p[j].ni = v.p[j].ti = 0.0f;
      v.p[j].rA = v.p[j].rB = zero2(); v.p[j].nm = v.p[j].tm = v.p[j].vb = 0.0f;
      v.lps[j] = zero2();
    }
    for (int j = 0; j < 2; ++j) {
      if (j >= ct.pointCount) break;
      if (warm) { v.p[j].ni = dtRatio * ct.pt[j].ni; v.p[j].ti = dtRatio * ct.pt[j].ti; }
      v.lps[j] = V(ct.pt[j].lx, ct.pt[j].ly);
    }
    VC_END(i);
  }
}

template <int NMAX> __device__ __forceinline__ void cs_init_velocity(VC* vc, int n, const Car& c, const BodyState& A) {
  const float mA = CAR_INV_MASS, iA = CAR_INV_I, mB = 0.0f, iB = 0.0f;
  const float friction_unused = 0.0f; (void)friction_unused;
  const Rot qA = rot_set(A.a);   // b2Rot::Set(aA) of every contact below: A is the same body state for all of them
#pragma unroll UNROLL_SMALL   // registers for small islands; the general bound stays a loop
  for (int i = 0; i < NMAX; ++i) {
    if (i >= n) break;
    VC_BEGIN(i);
    const DContact& m = c.ct[v.ci];
    V2 cA = A.c; float aA = A.a; V2 vA = A.v; float wA = A.w;
    V2 cB = v.cB; float aB = v.aB; V2 vB = v.vB; float wB = v.wB;
    Xf xfA, xfB;
    xfA.q = qA; xfB.q = rot_static(aB, v.aB0, v.qB);
    xfA.p = vsub(cA, rmul(xfA.q, zero2()));
    xfB.p = vsub(cB, rmul(xfB.q, zero2()));
    V2 normal = zero2(), pts[2];
    world_manifold(m, xfA, xfB, &normal, pts);
    v.normal = normal;
    for (int j = 0; j < 2; ++j) {
      if (j >= v.pointCount) break;
      VCP& p = v.p[j];
      p.rA = vsub(pts[j], cA); p.rB = vsub(pts[j], cB);
      float rnA = vcross(p.rA, v.normal), rnB = vcross(p.rB, v.normal);
      float kNormal = mA + mB + iA * rnA * rnA + iB * rnB * rnB;
      p.nm = kNormal > 0.0f ? fdiv_cr(1.0f, kNormal) : 0.0f;
      V2 tangent = vcross_vs(v.normal, 1.0f);
      float rtA = vcross(p.rA, tangent), rtB = vcross(p.rB, tangent);
      float kTangent = mA + mB + iA * rtA * rtA + iB * rtB * rtB;
      p.tm = kTangent > 0.0f ? fdiv_cr(1.0f, kTangent) : 0.0f;
      p.vb = 0.0f;
      float vRel = vdot(v.normal, vsub(vsub(vadd(vB, vcross_sv(wB, p.rB)), vA), vcross_sv(wA, p.rA)));
      if (vRel < -VELOCITY_THRESHOLD) p.vb = -MIX_RESTITUTION * vRel;
    }
    if (v.pointCount == 2) {
      VCP& p1 = v.p[0]; VCP& p2 = v.p[1];
      float rn1A = vcross(p1.rA, v.normal), rn1B = vcross(p1.rB, v.normal);
      float rn2A = vcross(p2.rA, v.normal), rn2B = vcross(p2.rB, v.normal);
      float k11 = mA + mB + iA * rn1A * rn1A + iB * rn1B * rn1B;
      float k22 = mA + mB + iA * rn2A * rn2A + iB * rn2B * rn2B;
      float k12 = mA + mB + iA * rn1A * rn2A + iB * rn1B * rn2B;
      if (k11 * k11 < 1000.0f * (k11 * k22 - k12 * k12)) {
        v.K[0] = k11; v.K[1] = k12; v.K[2] = k12; v.K[3] = k22;
        float a = v.K[0], b = v.K[2], cc = v.K[1], d = v.K[3];
        float det = a * d - b * cc;
        if (det != 0.0f) det = fdiv_cr(1.0f, det);
        v.nm[0] = det * d; v.nm[2] = -det * b; v.nm[1] = -det * cc; v.nm[3] = det * a;
      } else {
        v.pointCount = 1;
      }
    }
    VC_END(i);
  }
}

template <int NMAX> __device__ __forceinline__ void cs_warm_start(VC* vc, int n, BodyState& A) {
  const float mA = CAR_INV_MASS, iA = CAR_INV_I, mB = 0.0f, iB = 0.0f;
#pragma unroll UNROLL_SMALL   // registers for small islands; the general bound stays a loop
  for (int i = 0; i < NMAX; ++i) {
    if (i >= n) break;
    VC_BEGIN(i);
    V2 vA = A.v; float wA = A.w; V2 vB = v.vB; float wB = v.wB;
    V2 normal = v.normal, tangent = vcross_vs(normal, 1.0f);
    for (int j = 0; j < 2; ++j) {
      if (j >= v.pointCount) break;
      VCP& p = v.p[j];
      V2 P = vadd(vmul(p.ni, normal), vmul(p.ti, tangent));
      wA -= iA * vcross(p.rA, P);
      vA = vsub(vA, vmul(mA, P));
      wB += iB * vcross(p.rB, P);
      vB = vadd(vB, vmul(mB, P));
    }
    A.v = vA; A.w = wA; v.vB = vB; v.wB = wB;
    VC_END(i);
  }
}

__device__ __forceinline__ V2 rel_vel(V2 vA, float wA, V2 vB, float wB, const VCP& p) {
  return vsub(vsub(vadd(vB, vcross_sv(wB, p.rB)), vA), vcross_sv(wA, p.rA));
}

template <int NMAX> __device__ __forceinline__ void cs_solve_velocity(VC* vc, int n, BodyState& A, float friction) {
  const float mA = CAR_INV_MASS, iA = CAR_INV_I, mB = 0.0f, iB = 0.0f;
#pragma unroll UNROLL_SMALL   // registers for small islands; the general bound stays a loop
  for (int i = 0; i < NMAX; ++i) {
    if (i >= n) break;
    VC_BEGIN(i);
    V2 vA = A.v; float wA = A.w; V2 vB = v.vB; float wB = v.wB;
    V2 normal = v.normal, tangent = vcross_vs(normal, 1.0f);
    for (int j = 0; j < 2; ++j) {
      if (j >= v.pointCount) break;
      VCP& p = v.p[j];
      V2 dv = rel_vel(vA, wA, vB, wB, p);
      float vt = vdot(dv, tangent) - 0.0f;
      float lambda = p.tm * (-vt);
      float maxFriction = friction * p.ni;
      float newImpulse = fclamp(p.ti + lambda, -maxFriction, maxFriction);
      lambda = newImpulse - p.ti;
      p.ti = newImpulse;
      V2 P = vmul(lambda, tangent);
      vA = vsub(vA, vmul(mA, P)); wA -= iA * vcross(p.rA, P);
      vB = vadd(vB, vmul(mB, P)); wB += iB * vcross(p.rB, P);
    }
    if (v.pointCount == 1) {
      VCP& p = v.p[0];
      V2 dv = rel_vel(vA, wA, vB, wB, p);
      float vn = vdot(dv, normal);
      float lambda = -p.nm * (vn - p.vb);
      float newImpulse = fmaxb(p.ni + lambda, 0.0f);
      lambda = newImpulse - p.ni;
      p.ni = newImpulse;
      V2 P = vmul(lambda, normal);
      vA = vsub(vA, vmul(mA, P)); wA -= iA * vcross(p.rA, P);
      vB = vadd(vB, vmul(mB, P)); wB += iB * vcross(p.rB, P);
    } else {
      VCP& cp1 = v.p[0]; VCP& cp2 = v.p[1];
      V2 a = V(cp1.ni, cp2.ni);
      V2 dv1 = rel_vel(vA, wA, vB, wB, cp1), dv2 = rel_vel(vA, wA, vB, wB, cp2);
      float vn1 = vdot(dv1, normal), vn2 = vdot(dv2, normal);
      V2 b = V(vn1 - cp1.vb, vn2 - cp2.vb);
      V2 Ka = V(v.K[0] * a.x + v.K[2] * a.y, v.K[1] * a.x + v.K[3] * a.y);
      b = vsub(b, Ka);
      V2 x;
      bool ok = false;
      x = vneg(V(v.nm[0] * b.x + v.nm[2] * b.y, v.nm[1] * b.x + v.nm[3] * b.y));
      if (x.x >= 0.0f && x.y >= 0.0f) ok = true;
      if (!ok) {
        x.x = -cp1.nm * b.x; x.y = 0.0f;
        vn2 = v.K[1] * x.x + b.y;
        if (x.x >= 0.0f && vn2 >= 0.0f) ok = true;
      }
      if (!ok) {
        x.x = 0.0f; x.y = -cp2.nm * b.y;
        vn1 = v.K[2] * x.y + b.x;
        if (x.y >= 0.0f && vn1 >= 0.0f) ok = true;
      }
      if (!ok) {
        x.x = 0.0f; x.y = 0.0f; vn1 = b.x; vn2 = b.y;
        if (vn1 >= 0.0f && vn2 >= 0.0f) ok = true;
      }
      if (ok) {
        V2 d = vsub(x, a);
        V2 P1 = vmul(d.x, normal), P2 = vmul(d.y, normal);
        vA = vsub(vA, vmul(mA, vadd(P1, P2)));
        wA -= iA * (vcross(cp1.rA, P1) + vcross(cp2.rA, P2));
        vB = vadd(vB, vmul(mB, vadd(P1, P2)));
        wB += iB * (vcross(cp1.rB, P1) + vcross(cp2.rB, P2));
        cp1.ni = x.x; cp2.ni = x.y;
      }
    }
    A.v = vA; A.w = wA; v.vB = vB; v.wB = wB;
    VC_END(i);
  }
}

template <int NMAX> __device__ __forceinline__ void cs_store(const VC* vc, int n, Car& c) {
#pragma unroll UNROLL_SMALL   // registers for small islands; the general bound stays a loop
  for (int i = 0; i < NMAX; ++i) {
    if (i >= n) break;
    DContact& m = c.ct[vc[i].ci];
    for (int j = 0; j < 2; ++j) {
      if (j >= vc[i].pointCount) break; m.pt[j].ni = vc[i].p[j].ni; m.pt[j].ti = vc[i].p[j].ti; }
  }
}

// b2Rot::Set of the car's angle, recomputed only when the angle's bits changed since the last call (a point whose
// position impulse is zero leaves the angle bit for bit as it was: the same input, the same sinf / cosf)
struct RotCache { uint32_t bits; Rot q; };
__device__ __forceinline__ Rot rot_cached(RotCache& rc, float a) {
  if (__float_as_uint(a) != rc.bits) { rc.bits = __float_as_uint(a); rc.q = rot_set(a); }
  return rc.q;
}
template <int NMAX> __device__ __forceinline__ int cs_solve_position(VC* vc, int n, BodyState& A, int toi, RotCache& rcA) {
  float minSep = 0.0f;
  const float mA = CAR_INV_MASS, iA = CAR_INV_I, mB = 0.0f, iB = 0.0f;
#pragma unroll UNROLL_SMALL   // registers for small islands; the general bound stays a loop
  for (int i = 0; i < NMAX; ++i) {
    if (i >= n) break;
    VC_BEGIN(i);
    V2 cA = A.c; float aA = A.a; V2 cB = v.cB; float aB = v.aB;
    for (int j = 0; j < 2; ++j) {
      if (j >= v.pcount) break;
      Xf xfA, xfB;
      xfA.q = rot_cached(rcA, aA); xfB.q = rot_static(aB, v.aB0, v.qB);
      xfA.p = vsub(cA, rmul(xfA.q, zero2()));
      xfB.p = vsub(cB, rmul(xfB.q, zero2()));
      V2 normal, point; float sep;
      if (v.type == 1) {
        V2 nn = rmul(xfA.q, v.ln), planePoint = xmul(xfA, v.lp), clipPoint = xmul(xfB, v.lps[j]);
        sep = vdot(vsub(clipPoint, planePoint), nn) - POLY_RADIUS - POLY_RADIUS;
        point = clipPoint; normal = nn;
      } else {
        V2 nn = rmul(xfB.q, v.ln), planePoint = xmul(xfB, v.lp), clipPoint = xmul(xfA, v.lps[j]);
        sep = vdot(vsub(clipPoint, planePoint), nn) - POLY_RADIUS - POLY_RADIUS;
        point = clipPoint; normal = vneg(nn);
      }
      V2 rA = vsub(point, cA), rB = vsub(point, cB);
      minSep = fminb(minSep, sep);
      float C = fclamp((toi ? TOI_BAUMGARTE : BAUMGARTE) * (sep + LINEAR_SLOP), -MAX_LINEAR_CORRECTION, 0.0f);
      float rnA = vcross(rA, normal), rnB = vcross(rB, normal);
      float K = mA + mB + iA * rnA * rnA + iB * rnB * rnB;
      float impulse = K > 0.0f ? fdiv_cr(-C, K) : 0.0f;
      V2 P = vmul(impulse, normal);
      cA = vsub(cA, vmul(mA, P)); aA -= iA * vcross(rA, P);
      cB = vadd(cB, vmul(mB, P)); aB += iB * vcross(rB, P);
    }
    A.c = cA; A.a = aA; v.cB = cB; v.aB = aB;
    VC_END(i);
  }
  return toi ? (minSep >= -1.5f * LINEAR_SLOP) : (minSep >= -3.0f * LINEAR_SLOP);
}

template <int NMAX> __device__ __forceinline__ void report(Car& c, const VC* vc, int n) {
#pragma unroll UNROLL_SMALL   // registers for small islands; the general bound stays a loop
  for (int i = 0; i < NMAX; ++i) {
    if (i >= n) break;
    lis_post(c, vc[i].pointCount, vc[i].p[0].ni, vc[i].p[1].ni);
  }
}

__device__ inline void integrate_positions(BodyState& A, float h) {
  V2 cc = A.c; float a = A.a; V2 v = A.v; float w = A.w;
  V2 translation = vmul(h, v);
  if (vdot(translation, translation) > MAX_TRANSLATION * MAX_TRANSLATION) {
    float ratio = fdiv_cr(MAX_TRANSLATION, vlen(translation));
    v = vmul(ratio, v);
  }
  float rotation = h * w;
  if (rotation * rotation > MAX_ROTATION * MAX_ROTATION) {
    float ratio = fdiv_cr(MAX_ROTATION, fabsf(rotation));
    w *= ratio;
  }
  cc = vadd(cc, vmul(h, v));
  a += h * w;
  A.c = cc; A.a = a; A.v = v; A.w = w;
}

// island contact list: cidx[n] = i without a dynamically indexed store (selects keep cidx in registers)
__device__ __forceinline__ void island_push(int cidx[MAX_ISLAND], int& n, int i) {
#pragma unroll
  for (int j = 0; j < MAX_ISLAND; ++j) cidx[j] = j == n ? i : cidx[j];
  ++n;
}
// the island solve of b2World::Solve for n touching contacts; NMAX >= n contact constraints in registers (the
// common islands of 1-2 contacts; a larger bound would sit in scratch memory)
template <int NMAX>
__device__ __forceinline__ int solve_island_buf(Car& c, const LWall* W, const int* cidx, int n, float dt, float dtRatio,
                                                float friction, VC* vc) {
  float h = dt;
  BodyState A;
  c.c0 = c.c; c.a0 = c.a;
  {
    V2 v = c.v; float wv = c.w;
    V2 g = vadd(vmul(1.0f, zero2()), vmul(CAR_INV_MASS, c.force));
    v = vadd(v, vmul(h, g));
    wv += h * CAR_INV_I * c.torque;
    A.c = c.c; A.a = c.a; A.v = v; A.w = wv;
  }
  cs_init<NMAX>(vc, n, c, cidx, W, true, dtRatio);
  cs_init_velocity<NMAX>(vc, n, c, A);
  cs_warm_start<NMAX>(vc, n, A);
  SOLVER_ITER_LOOP
  for (int it = 0; it < 6; ++it) cs_solve_velocity<NMAX>(vc, n, A, friction);
  cs_store<NMAX>(vc, n, c);
  integrate_positions(A, h);
  int positionSolved = 0;
  RotCache rcA; rcA.bits = __float_as_uint(A.a) ^ 1u; rcA.q.s = 0.0f; rcA.q.c = 1.0f;   // (empty: no angle matches)
  SOLVER_ITER_LOOP
  for (int it = 0; it < 4; ++it) { if (cs_solve_position<NMAX>(vc, n, A, 0, rcA)) { positionSolved = 1; break; } }
  c.c = A.c; c.a = A.a; c.v = A.v; c.w = A.w;
  c.xf.q = rot_cached(rcA, c.a); c.xf.p = vsub(c.c, rmul(c.xf.q, zero2()));   // sync_transform
  report<NMAX>(c, vc, n);
  return positionSolved;
}
template <int NMAX>
__device__ __forceinline__ int solve_island(Car& c, const LWall* W, const int* cidx, int n, float dt, float dtRatio,
                                            float friction) {
  VC vc[NMAX];   // small islands: fully unrolled, register-resident
  return solve_island_buf<NMAX>(c, W, cidx, n, dt, dtRatio, friction, vc);
}
// The general island (more than ISLAND_MID touching contacts) indexes its constraints dynamically; as a private
// array they would live in scratch memory (1.6 KB per lane, a vector-memory round trip per field use).  Instead
// the wave's LDS work area (free during b2World::Solve and an event's island solve) holds them, one lane at a time
// -- the lowest lane of the wave still waiting goes next.  Divergent lanes of a wave run one after another anyway,
// so serialising them costs nothing over the private-array form; every access is an LDS round trip.
#ifndef ISLAND_LDS
#define ISLAND_LDS 1
#endif
template <typename F>
__device__ __forceinline__ void wave_lds_one_at_a_time(F&& body) {
  unsigned long long pending = __ballot(1);   // the lanes of this wave executing this call
  wave_lds_sync();                            // earlier LDS reads of the work area (any lane) done before its reuse
  while (pending) {                           // wave-uniform
    const int leader = __ffsll((long long)pending) - 1;
    if ((int)__lane_id() == leader) body((VC*)g_wave_lds[threadIdx.x >> 6].island.vc);
    pending &= pending - 1;
    wave_lds_sync();
  }
}
__device__ __forceinline__ int solve_island_general(Car& c, const LWall* W, const int* cidx, int n, float dt,
                                                   float dtRatio, float friction) {
#if ISLAND_LDS
  int r = 0;
  wave_lds_one_at_a_time([&](VC* vc) { r = solve_island_buf<MAX_ISLAND>(c, W, cidx, n, dt, dtRatio, friction, vc); });
  return r;
#else
  return solve_island<MAX_ISLAND>(c, W, cidx, n, dt, dtRatio, friction);
#endif
}

// b2BroadPhase::UpdatePairs of b2World::Solve for every lane of the wave at once (round 3).  A moved car's grid
// cell lists its candidate walls in ascending proxy id; here every present lane tests any (car, candidate) pair of
// the wave -- the candidate's fat AABB against the owner's, read from LDS -- and sets the pair's bit in the owner's
// hit mask, then each owner runs AddPair for its hits in ascending candidate order: the same pairs in the same
// order as find_new_contacts' own loop, with one round of independent loads per wave instead of a dependent chain
// per car.  Lists longer than 64 candidates, queries outside the grid or wider than its reach take the car's own scan.
#ifndef BP_COOP
#define BP_COOP 0   // measured neutral (160.7 vs 159.2 us/step, 3 A/B rounds): the broadphase chain is not its candidate loads
#endif
#ifndef MODEL_PRIO
#define MODEL_PRIO 0   // wave priority experiments (0: off)
#endif
__device__ inline void find_new_contacts_wave(Car& c, const WallSet& S, bool want) {
  bool mine = false; int beg = 0, end = 0;
  if (want && c.moved) {
    const float hx = 0.5f * (c.fat.hi.x - c.fat.lo.x), hy = 0.5f * (c.fat.hi.y - c.fat.lo.y);
    const float cx = 0.5f * (c.fat.hi.x + c.fat.lo.x), cy = 0.5f * (c.fat.hi.y + c.fat.lo.y);
    if (S.bp.box && hx <= S.bp.reach - 0.05f && hy <= S.bp.reach - 0.05f && grid_list(S.bp, cx, cy, beg, end) &&
        end - beg <= 64) {
      mine = true;
      c.moved = 0;
    } else {
      find_new_contacts(c, S);
    }
  }
  if (!__ballot(mine)) return;   // wave-uniform
  BpWaveLDS& B = g_wave_lds[threadIdx.x >> 6].bp;
  const int lane = (int)__lane_id();
  const unsigned long long present = __ballot(1);
  const int prank = rank_in(present), npresent = popc64(present);
  const int m = mine ? end - beg : 0;
  int off = 0, total = 0;
#pragma unroll
  for (int bit = 0; bit < 7; ++bit) {
    const unsigned long long b = __ballot((m >> bit) & 1);
    off += rank_in(b) << bit;
    total += popc64(b) << bit;
  }
  if (mine) { B.fat[lane] = make_float4(c.fat.lo.x, c.fat.lo.y, c.fat.hi.x, c.fat.hi.y); B.hit[lane][0] = 0u; B.hit[lane][1] = 0u; }
  for (int r0 = 0; r0 < total; r0 += BP_JOBCAP) {   // wave-uniform
    if (mine) {
      const int k1 = min(off + m, r0 + BP_JOBCAP);
      for (int k = max(off, r0); k < k1; ++k) B.job[k - r0] = make_int2(lane | ((k - off) << 8), beg + (k - off));
    }
    wave_lds_sync();
    const int cnt = min(BP_JOBCAP, total - r0);
    for (int j = prank; j < cnt; j += npresent) {
      const int2 jb = B.job[j];
      const int owner = jb.x & 0xFF, q = jb.x >> 8;
      const float4 f = B.fat[owner], b = ldg(S.bp.box + jb.y);
      Aabb fa; fa.lo = V(f.x, f.y); fa.hi = V(f.z, f.w);
      Aabb bb; bb.lo = V(b.x, b.y); bb.hi = V(b.z, b.w);
      if (overlap(fa, bb)) atomicOr(&B.hit[owner][q >> 5], 1u << (q & 31));
    }
    wave_lds_sync();
  }
  if (mine) {
    unsigned long long h = (unsigned long long)B.hit[lane][0] | ((unsigned long long)B.hit[lane][1] << 32);
    while (h) {
      const int q = __ffsll((long long)h) - 1; h &= h - 1;
      add_pair(c, S, (int)ldg(S.bp.idx + beg + q));
    }
  }
  wave_lds_sync();   // hit masks read before the union's next use
}

// b2World::Solve (single dynamic body island)
__device__ inline void solve(Car& c, const WallSet& S, float dt, float dtRatio, float friction) {
  const LWall* W = S.W;
  if (!c.awake) return;
  int cidx[MAX_ISLAND] = {0, 0, 0, 0, 0, 0, 0, 0}; int n = 0;
  for (int i = 0; i < c.nct; ++i) {
    int fl = c.ct[i].flags;
    if (!(fl & CT_ENABLED) || !(fl & CT_TOUCH)) continue;
    if (n == MAX_ISLAND) { c.overflow = 2; break; }
    island_push(cidx, n, i);
  }
  const float h = dt;
  CCOUNT(c, 26, n);   // profile builds: the island's touching contacts and its solve cycles (slot 25)
  CTIME_BEGIN();
#if ISLAND_MID
  const int positionSolved = n <= ISLAND_TWO ? solve_island<2>(c, W, cidx, n, dt, dtRatio, friction)
                           : n <= ISLAND_MID ? solve_island<ISLAND_MID>(c, W, cidx, n, dt, dtRatio, friction)
                                             : solve_island_general(c, W, cidx, n, dt, dtRatio, friction);
#else
  const int positionSolved = n <= 2 ? solve_island<2>(c, W, cidx, n, dt, dtRatio, friction)
                                    : solve_island<MAX_ISLAND>(c, W, cidx, n, dt, dtRatio, friction);
#endif
  CTIME_END(c, 25);
  {
    float minSleepTime = FLT_BIG;
    const float linTolSqr = LINEAR_SLEEP_TOL * LINEAR_SLEEP_TOL;
    const float angTolSqr = ANGULAR_SLEEP_TOL * ANGULAR_SLEEP_TOL;
    if (c.w * c.w > angTolSqr || vdot(c.v, c.v) > linTolSqr) { c.sleep = 0.0f; minSleepTime = 0.0f; }
    else { c.sleep += h; minSleepTime = fminb(minSleepTime, c.sleep); }
    if (minSleepTime >= TIME_TO_SLEEP && positionSolved) {
      c.awake = 0; c.sleep = 0.0f; c.v = zero2(); c.w = 0.0f; c.force = zero2(); c.torque = 0.0f;
    }
  }
  PROFB(12);
  {
  CTIME_BEGIN();
  sync_fixtures(c);
  CTIME_END(c, 22);
  }
#if !BP_COOP   // (else b2_step runs the wave's broadphase updates together: find_new_contacts_wave)
  {
  CTIME_BEGIN();
  if (c.moved) CCOUNT(c, 24, 1);
  find_new_contacts(c, S);
  CTIME_END(c, 21);
  }
#endif
}

// ------------------------------------------------------------------ GJK / TOI
// b2Distance (GJK) with the simplex vertices and the cache indices as named values (no dynamically indexed
// arrays: those lived in scratch memory).  Same operations in the same order as b2Simplex::ReadCache /
// Solve2 / Solve3 / GetSearchDirection / GetWitnessPoints / WriteCache.
struct SV { V2 wA, wB, w; float a; int iA, iB; };
struct SCache { float metric; int count; int iA0, iA1, iA2, iB0, iB1, iB2;
#ifdef NASCAR_PROFILE
  int iters = 0;   // profile builds: GJK iterations summed over the calls that used this cache
#endif
};

#ifndef SUPPORT_BOX
#define SUPPORT_BOX 1
#endif
// b2PolygonShape / b2DistanceProxy::GetSupport: the first vertex of maximal dot product with d.  For a box the four
// dot products (+-hx) dx + (+-hy) dy share the two products a = hx dx, b = hy dy ((-hx) dx is -(hx dx) exactly in
// IEEE arithmetic), so they are (-a) + (-b), a + (-b), a + b, (-a) + b -- the same values, 2 products instead of 8.
__device__ __forceinline__ int support(const Poly* p, V2 d) {
#if SUPPORT_BOX
  const float a = p->hx * d.x, b = p->hy * d.y;
  const float v1 = a + (-b), v2 = a + b, v3 = (-a) + b;
  int best = 0; float bestValue = (-a) + (-b);
  if (v1 > bestValue) { best = 1; bestValue = v1; }
  if (v2 > bestValue) { best = 2; bestValue = v2; }
  if (v3 > bestValue) { best = 3; }
  return best;
#else
  int best = 0; float bestValue = vdot(pv(p, 0), d);
  for (int i = 1; i < 4; ++i) { float value = vdot(pv(p, i), d); if (value > bestValue) { best = i; bestValue = value; } }
  return best;
#endif
}
__device__ __forceinline__ float simplex_metric(int count, const SV& v0, const SV& v1, const SV& v2) {
  if (count == 1) return 0.0f;
  if (count == 2) return vlen(vsub(v0.w, v1.w));
  if (count == 3) return vcross(vsub(v1.w, v0.w), vsub(v2.w, v0.w));
  return 0.0f;
}
__device__ __forceinline__ void sv_set(SV& v, int ia, int ib, const Poly* pA, Xf tA, const Poly* pB, Xf tB) {
  v.iA = ia; v.iB = ib;
  v.wA = xmul(tA, pv(pA, ia)); v.wB = xmul(tB, pv(pB, ib));
  v.w = vsub(v.wB, v.wA); v.a = 0.0f;
}
#ifndef GJK_V2
#define GJK_V2 1
#endif
#if GJK_V2
// b2Distance (b2GJK) for two boxes, restated for a short dependent chain: the simplex is held as its vertices' w
// (= wB - wA), packed index pairs (iA | iB << 2) and barycentric weights only -- the support points wA / wB are
// recomputed from their indices where b2Simplex::GetWitnessPoints needs them (b2Transform * vertex again: the same
// operations on the same values) -- and Solve2 / Solve3's case analysis is evaluated as selects with one division
// (the chosen case's denominator), so a step moves 5 registers per vertex instead of 9 and takes no branch per case.
// Same cases in the same priority order, same arithmetic per case: identical results (tools/toi_bench.py compares the
// alphas of the captured steady-state TOI jobs bit for bit; the GPU parity suite covers the rest).
__device__ __forceinline__ V2 gjk_w(int ip, const Poly* pA, Xf tA, const Poly* pB, Xf tB) {
  return vsub(xmul(tB, pv(pB, ip >> 2)), xmul(tA, pv(pA, ip & 3)));
}
__device__ inline float gjk_distance(SCache& cache, const Poly* pA, Xf tA, const Poly* pB, Xf tB) {
  V2 w0 = zero2(), w1 = zero2(), w2 = zero2();
  int i0 = 0, i1 = 0, i2 = 0;
  float a0 = 0.0f, a1 = 0.0f, a2 = 0.0f;
  int count = cache.count;
  if (count > 0) { i0 = cache.iA0 | (cache.iB0 << 2); w0 = gjk_w(i0, pA, tA, pB, tB); }
  if (count > 1) { i1 = cache.iA1 | (cache.iB1 << 2); w1 = gjk_w(i1, pA, tA, pB, tB); }
  if (count > 2) { i2 = cache.iA2 | (cache.iB2 << 2); w2 = gjk_w(i2, pA, tA, pB, tB); }
  if (count > 1) {   // b2Simplex::ReadCache: flush a cache whose metric changed a lot
    const float metric1 = cache.metric;
    const float metric2 = count == 2 ? vlen(vsub(w0, w1)) : (count == 3 ? vcross(vsub(w1, w0), vsub(w2, w0)) : 0.0f);
    if (metric2 < 0.5f * metric1 || 2.0f * metric1 < metric2 || metric2 < FLT_EPS) count = 0;
  }
  if (count == 0) { i0 = 0; w0 = gjk_w(0, pA, tA, pB, tB); a0 = 1.0f; count = 1; }
  int iter = 0;
  while (iter < 20) {
    const int saveCount = count, s0 = i0, s1 = i1, s2 = i2;
    if (count == 2) {   // b2Simplex::Solve2
      const V2 e12 = vsub(w1, w0);
      const float d12_2 = -vdot(w0, e12), d12_1 = vdot(w1, e12);
      const bool c1 = d12_2 <= 0.0f, c2 = !c1 && d12_1 <= 0.0f, c3 = !c1 && !c2;
      const float inv = fdiv_cr(1.0f, c3 ? d12_1 + d12_2 : 1.0f);
      if (c2) { w0 = w1; i0 = i1; }
      a0 = c3 ? d12_1 * inv : 1.0f;
      a1 = c3 ? d12_2 * inv : (c2 ? 1.0f : a1);
      count = c3 ? 2 : 1;
    } else if (count == 3) {   // b2Simplex::Solve3
      const V2 e12 = vsub(w1, w0);
      const float d12_1 = vdot(w1, e12), d12_2 = -vdot(w0, e12);
      const V2 e13 = vsub(w2, w0);
      const float d13_1 = vdot(w2, e13), d13_2 = -vdot(w0, e13);
      const V2 e23 = vsub(w2, w1);
      const float d23_1 = vdot(w2, e23), d23_2 = -vdot(w1, e23);
      const float n123 = vcross(e12, e13);
      const float d123_1 = n123 * vcross(w1, w2), d123_2 = n123 * vcross(w2, w0), d123_3 = n123 * vcross(w0, w1);
      const bool cA = d12_2 <= 0.0f && d13_2 <= 0.0f;
      const bool cB = !cA && d12_1 > 0.0f && d12_2 > 0.0f && d123_3 <= 0.0f;
      const bool cC = !cA && !cB && d13_1 > 0.0f && d13_2 > 0.0f && d123_2 <= 0.0f;
      const bool cD = !cA && !cB && !cC && d12_1 <= 0.0f && d23_2 <= 0.0f;
      const bool cE = !cA && !cB && !cC && !cD && d13_1 <= 0.0f && d23_1 <= 0.0f;
      const bool cF = !cA && !cB && !cC && !cD && !cE && d23_1 > 0.0f && d23_2 > 0.0f && d123_1 <= 0.0f;
      const bool cG = !cA && !cB && !cC && !cD && !cE && !cF;
      const float den = cB ? d12_1 + d12_2 : cC ? d13_1 + d13_2 : cF ? d23_1 + d23_2 : cG ? d123_1 + d123_2 + d123_3 : 1.0f;
      const float inv = fdiv_cr(1.0f, den);
      // new vertex 0: old 0 (A, B, C, G), old 1 (D), old 2 (E, F); new vertex 1: old 2 (C), else old 1
      const V2 n0 = cD ? w1 : (cE || cF) ? w2 : w0;
      const int j0 = cD ? i1 : (cE || cF) ? i2 : i0;
      const float b0 = cB ? d12_1 * inv : cC ? d13_1 * inv : cF ? d23_2 * inv : cG ? d123_1 * inv : 1.0f;
      const float b1 = cB ? d12_2 * inv : cC ? d13_2 * inv : cF ? d23_1 * inv : cG ? d123_2 * inv : cD ? 1.0f : a1;
      if (cC) { w1 = w2; i1 = i2; }
      w0 = n0; i0 = j0; a0 = b0; a1 = b1;
      if (cG) a2 = d123_3 * inv;
      else if (cE) a2 = 1.0f;
      else if (cC) a2 = d13_2 * inv;
      else if (cF) a2 = d23_2 * inv;
      count = cG ? 3 : (cB || cC || cF) ? 2 : 1;
    }
    if (count == 3) break;
    V2 d;
    if (count == 1) d = vneg(w0);
    else {
      const V2 e12 = vsub(w1, w0);
      const float sgn = vcross(e12, vneg(w0));
      d = sgn > 0.0f ? vcross_sv(1.0f, e12) : vcross_vs(e12, 1.0f);
    }
    if (vdot(d, d) < FLT_EPS * FLT_EPS) break;
    const int ia = support(pA, rmulT(tA.q, vneg(d)));
    const int ib = support(pB, rmulT(tB.q, d));
    const int ix = ia | (ib << 2);
    const V2 wx = vsub(xmul(tB, pv(pB, ib)), xmul(tA, pv(pA, ia)));
    ++iter;
#ifdef NASCAR_PROFILE
    ++cache.iters;
#endif
    const bool dup = ix == s0 || (saveCount > 1 && ix == s1) || (saveCount > 2 && ix == s2);
    if (dup) break;
    if (count == 1) { w1 = wx; i1 = ix; a1 = 0.0f; } else { w2 = wx; i2 = ix; a2 = 0.0f; }
    ++count;
  }
  // b2Simplex::GetWitnessPoints, the support points recomputed from their indices
  V2 wa = zero2(), wb = zero2();
  const V2 wA0 = xmul(tA, pv(pA, i0 & 3)), wB0 = xmul(tB, pv(pB, i0 >> 2));
  if (count == 1) { wa = wA0; wb = wB0; }
  else {
    const V2 wA1 = xmul(tA, pv(pA, i1 & 3)), wB1 = xmul(tB, pv(pB, i1 >> 2));
    if (count == 2) {
      wa = vadd(vmul(a0, wA0), vmul(a1, wA1));
      wb = vadd(vmul(a0, wB0), vmul(a1, wB1));
    } else if (count == 3) {
      const V2 wA2 = xmul(tA, pv(pA, i2 & 3));
      wa = vadd(vadd(vmul(a0, wA0), vmul(a1, wA1)), vmul(a2, wA2));
      wb = wa;
    }
  }
  cache.metric = count == 2 ? vlen(vsub(w0, w1)) : (count == 3 ? vcross(vsub(w1, w0), vsub(w2, w0)) : 0.0f);
  cache.count = count;
  cache.iA0 = i0 & 3; cache.iB0 = i0 >> 2; cache.iA1 = i1 & 3; cache.iB1 = i1 >> 2; cache.iA2 = i2 & 3; cache.iB2 = i2 >> 2;
  return vlen(vsub(wa, wb));
}
#else
__device__ inline float gjk_distance(SCache& cache, const Poly* pA, Xf tA, const Poly* pB, Xf tB) {
  SV v0, v1, v2;
  v0.wA = v0.wB = v0.w = zero2(); v0.a = 0.0f; v0.iA = v0.iB = 0;
  v2 = v1 = v0;
  int count = cache.count;
  if (count > 0) sv_set(v0, cache.iA0, cache.iB0, pA, tA, pB, tB);
  if (count > 1) sv_set(v1, cache.iA1, cache.iB1, pA, tA, pB, tB);
  if (count > 2) sv_set(v2, cache.iA2, cache.iB2, pA, tA, pB, tB);
  if (count > 1) {
    float metric1 = cache.metric, metric2 = simplex_metric(count, v0, v1, v2);
    if (metric2 < 0.5f * metric1 || 2.0f * metric1 < metric2 || metric2 < FLT_EPS) count = 0;
  }
  if (count == 0) {
    sv_set(v0, 0, 0, pA, tA, pB, tB);
    v0.a = 1.0f;
    count = 1;
  }
  int sA0 = 0, sA1 = 0, sA2 = 0, sB0 = 0, sB1 = 0, sB2 = 0, saveCount = 0, iter = 0;
  while (iter < 20) {
    saveCount = count;
    sA0 = v0.iA; sB0 = v0.iB; sA1 = v1.iA; sB1 = v1.iB; sA2 = v2.iA; sB2 = v2.iB;
    if (count == 2) {
      V2 w1 = v0.w, w2 = v1.w, e12 = vsub(w2, w1);
      float d12_2 = -vdot(w1, e12);
      if (d12_2 <= 0.0f) { v0.a = 1.0f; count = 1; }
      else {
        float d12_1 = vdot(w2, e12);
        if (d12_1 <= 0.0f) { v1.a = 1.0f; count = 1; v0 = v1; }
        else { float inv = fdiv_cr(1.0f, d12_1 + d12_2); v0.a = d12_1 * inv; v1.a = d12_2 * inv; count = 2; }
      }
    } else if (count == 3) {
      V2 w1 = v0.w, w2 = v1.w, w3 = v2.w;
      V2 e12 = vsub(w2, w1);
      float d12_1 = vdot(w2, e12), d12_2 = -vdot(w1, e12);
      V2 e13 = vsub(w3, w1);
      float d13_1 = vdot(w3, e13), d13_2 = -vdot(w1, e13);
      V2 e23 = vsub(w3, w2);
      float d23_1 = vdot(w3, e23), d23_2 = -vdot(w2, e23);
      float n123 = vcross(e12, e13);
      float d123_1 = n123 * vcross(w2, w3), d123_2 = n123 * vcross(w3, w1), d123_3 = n123 * vcross(w1, w2);
      if (d12_2 <= 0.0f && d13_2 <= 0.0f) { v0.a = 1.0f; count = 1; }
      else if (d12_1 > 0.0f && d12_2 > 0.0f && d123_3 <= 0.0f) {
        float inv = fdiv_cr(1.0f, d12_1 + d12_2); v0.a = d12_1 * inv; v1.a = d12_2 * inv; count = 2;
      } else if (d13_1 > 0.0f && d13_2 > 0.0f && d123_2 <= 0.0f) {
        float inv = fdiv_cr(1.0f, d13_1 + d13_2); v0.a = d13_1 * inv; v2.a = d13_2 * inv; count = 2; v1 = v2;
      } else if (d12_1 <= 0.0f && d23_2 <= 0.0f) { v1.a = 1.0f; count = 1; v0 = v1; }
      else if (d13_1 <= 0.0f && d23_1 <= 0.0f) { v2.a = 1.0f; count = 1; v0 = v2; }
      else if (d23_1 > 0.0f && d23_2 > 0.0f && d123_1 <= 0.0f) {
        float inv = fdiv_cr(1.0f, d23_1 + d23_2); v1.a = d23_1 * inv; v2.a = d23_2 * inv; count = 2; v0 = v2;
      } else {
        float inv = fdiv_cr(1.0f, d123_1 + d123_2 + d123_3);
        v0.a = d123_1 * inv; v1.a = d123_2 * inv; v2.a = d123_3 * inv; count = 3;
      }
    }
    if (count == 3) break;
    V2 d;
    if (count == 1) d = vneg(v0.w);
    else {
      V2 e12 = vsub(v1.w, v0.w);
      float sgn = vcross(e12, vneg(v0.w));
      d = sgn > 0.0f ? vcross_sv(1.0f, e12) : vcross_vs(e12, 1.0f);
    }
    if (vdot(d, d) < FLT_EPS * FLT_EPS) break;
    SV vx;
    vx.iA = support(pA, rmulT(tA.q, vneg(d)));
    vx.wA = xmul(tA, pv(pA, vx.iA));
    vx.iB = support(pB, rmulT(tB.q, d));
    vx.wB = xmul(tB, pv(pB, vx.iB));
    vx.w = vsub(vx.wB, vx.wA);
    vx.a = 0.0f;
    ++iter;
#ifdef NASCAR_PROFILE
    ++cache.iters;
#endif
    bool dup = (vx.iA == sA0 && vx.iB == sB0) || (saveCount > 1 && vx.iA == sA1 && vx.iB == sB1) ||
               (saveCount > 2 && vx.iA == sA2 && vx.iB == sB2);
    if (dup) break;
    if (count == 1) v1 = vx; else v2 = vx;
    ++count;
  }
  V2 wa = zero2(), wb = zero2();
  if (count == 1) { wa = v0.wA; wb = v0.wB; }
  else if (count == 2) {
    wa = vadd(vmul(v0.a, v0.wA), vmul(v1.a, v1.wA));
    wb = vadd(vmul(v0.a, v0.wB), vmul(v1.a, v1.wB));
  } else if (count == 3) {
    wa = vadd(vadd(vmul(v0.a, v0.wA), vmul(v1.a, v1.wA)), vmul(v2.a, v2.wA));
    wb = wa;
  }
  cache.metric = simplex_metric(count, v0, v1, v2);
  cache.count = count;
  cache.iA0 = v0.iA; cache.iB0 = v0.iB; cache.iA1 = v1.iA; cache.iB1 = v1.iB; cache.iA2 = v2.iA; cache.iB2 = v2.iB;
  return vlen(vsub(wa, wb));
}

#endif

struct Sweep { V2 c0, c; float a0, a, alpha0; };
__device__ __forceinline__ Xf sweep_xf(const Sweep& s, float beta) {
  Xf xf;
  xf.p = vadd(vmul(1.0f - beta, s.c0), vmul(beta, s.c));
  float angle = (1.0f - beta) * s.a0 + beta * s.a;
  xf.q = rot_set(angle);
  xf.p = vsub(xf.p, rmul(xf.q, zero2()));
  return xf;
}
// b2Sweep::GetTransform of a static body's sweep (c0 == c, a0 == a): the interpolated angle is usually a0
// again, and then its rotation is q0 (rot_set(a0), computed once per TOI call) -- same values, one sincos less
__device__ __forceinline__ Xf sweep_xf_static(const Sweep& s, float beta, Rot q0) {
  Xf xf;
  xf.p = vadd(vmul(1.0f - beta, s.c0), vmul(beta, s.c));
  float angle = (1.0f - beta) * s.a0 + beta * s.a;
  xf.q = angle == s.a0 ? q0 : rot_set(angle);
  xf.p = vsub(xf.p, rmul(xf.q, zero2()));
  return xf;
}
__device__ __forceinline__ void sweep_normalize(Sweep& s) {
  float twoPi = 2.0f * B2_PI;
  float d = twoPi * floorf(fdiv_cr(s.a0, twoPi));
  s.a0 -= d; s.a -= d;
}

enum { SF_POINTS, SF_FACEA, SF_FACEB };
// body B (the wall) is static in every TOI here: its sweep transforms go through sweep_xf_static with qB
struct SepFn { Sweep sA, sB; Rot qB; int type; V2 lp, axis; };
// xfA / xfB: the sweeps' transforms at t1 (the caller's, computed once per b2TimeOfImpact iteration)
__device__ inline void sep_init(SepFn& f, const SCache& cache, const Poly* pA, const Sweep& sA, const Poly* pB, const Sweep& sB,
                                Rot qB, Xf xfA, Xf xfB) {
  f.sA = sA; f.sB = sB; f.qB = qB;
  if (cache.count == 1) {
    f.type = SF_POINTS;
    V2 pointA = xmul(xfA, pv(pA, cache.iA0)), pointB = xmul(xfB, pv(pB, cache.iB0));
    f.axis = vsub(pointB, pointA);
    vnormalize(&f.axis);
    f.lp = zero2();
  } else if (cache.iA0 == cache.iA1) {
    f.type = SF_FACEB;
    V2 lB1 = pv(pB, cache.iB0), lB2 = pv(pB, cache.iB1);
    f.axis = vcross_vs(vsub(lB2, lB1), 1.0f);
    vnormalize(&f.axis);
    V2 normal = rmul(xfB.q, f.axis);
    f.lp = vmul(0.5f, vadd(lB1, lB2));
    V2 pointB = xmul(xfB, f.lp), pointA = xmul(xfA, pv(pA, cache.iA0));
    float s = vdot(vsub(pointA, pointB), normal);
    if (s < 0.0f) f.axis = vneg(f.axis);
  } else {
    f.type = SF_FACEA;
    V2 lA1 = pv(pA, cache.iA0), lA2 = pv(pA, cache.iA1);
    f.axis = vcross_vs(vsub(lA2, lA1), 1.0f);
    vnormalize(&f.axis);
    V2 normal = rmul(xfA.q, f.axis);
    f.lp = vmul(0.5f, vadd(lA1, lA2));
    V2 pointA = xmul(xfA, f.lp), pointB = xmul(xfB, pv(pB, cache.iB0));
    float s = vdot(vsub(pointB, pointA), normal);
    if (s < 0.0f) f.axis = vneg(f.axis);
  }
}
// b2SeparationFunction::FindMinSeparation / Evaluate on the sweeps' transforms at t (xfA, xfB)
__device__ inline float sep_find_min(const SepFn& f, const Poly* pA, const Poly* pB, int* iA, int* iB, Xf xfA, Xf xfB) {
  if (f.type == SF_POINTS) {
    V2 axisA = rmulT(xfA.q, f.axis), axisB = rmulT(xfB.q, vneg(f.axis));
    *iA = support(pA, axisA); *iB = support(pB, axisB);
    V2 pointA = xmul(xfA, pv(pA, *iA)), pointB = xmul(xfB, pv(pB, *iB));
    return vdot(vsub(pointB, pointA), f.axis);
  } else if (f.type == SF_FACEA) {
    V2 normal = rmul(xfA.q, f.axis), pointA = xmul(xfA, f.lp);
    V2 axisB = rmulT(xfB.q, vneg(normal));
    *iA = -1; *iB = support(pB, axisB);
    V2 pointB = xmul(xfB, pv(pB, *iB));
    return vdot(vsub(pointB, pointA), normal);
  } else {
    V2 normal = rmul(xfB.q, f.axis), pointB = xmul(xfB, f.lp);
    V2 axisA = rmulT(xfA.q, vneg(normal));
    *iB = -1; *iA = support(pA, axisA);
    V2 pointA = xmul(xfA, pv(pA, *iA));
    return vdot(vsub(pointA, pointB), normal);
  }
}
__device__ inline float sep_eval(const SepFn& f, const Poly* pA, const Poly* pB, int iA, int iB, Xf xfA, Xf xfB) {
  if (f.type == SF_POINTS) {
    V2 pointA = xmul(xfA, pv(pA, iA)), pointB = xmul(xfB, pv(pB, iB));
    return vdot(vsub(pointB, pointA), f.axis);
  } else if (f.type == SF_FACEA) {
    V2 normal = rmul(xfA.q, f.axis), pointA = xmul(xfA, f.lp), pointB = xmul(xfB, pv(pB, iB));
    return vdot(vsub(pointB, pointA), normal);
  } else {
    V2 normal = rmul(xfB.q, f.axis), pointB = xmul(xfB, f.lp), pointA = xmul(xfA, pv(pA, iA));
    return vdot(vsub(pointA, pointB), normal);
  }
}
enum { TOI_UNKNOWN, TOI_FAILED, TOI_OVERLAPPED, TOI_TOUCHING, TOI_SEPARATED };
// qB0 / aB0: the static body B's rotation and the angle bits it was set from (its body transform): b2Rot::Set of
// B's normalized sweep angle is that rotation whenever the normalization left the angle unchanged
__device__ inline float time_of_impact(int* state, const Poly* pA, const Sweep& sweepA, const Poly* pB, const Sweep& sweepB, float tMax,
                                      Rot qB0, uint32_t aB0, int* prof_iters = nullptr, unsigned long long* prof_cyc = nullptr) {
  *state = TOI_UNKNOWN;
  float out_t = tMax;
  Sweep sA = sweepA, sB = sweepB;
  sweep_normalize(sA); sweep_normalize(sB);
  const Rot qB = rot_static(sB.a0, aB0, qB0);
  float totalRadius = pA->radius + pB->radius;
  float target = fmaxb(LINEAR_SLOP, totalRadius - 3.0f * LINEAR_SLOP);
  float tolerance = 0.25f * LINEAR_SLOP;
  float t1 = 0.0f;
  int iter = 0;
  SCache cache; cache.count = 0; cache.metric = 0.0f;
  cache.iA0 = cache.iA1 = cache.iA2 = cache.iB0 = cache.iB1 = cache.iB2 = 0;
  Xf xfA = sweep_xf(sA, t1), xfB = sweep_xf_static(sB, t1, qB);   // at t1; carried over when t1 takes t2's value
  for (;;) {
#ifdef NASCAR_PROFILE
    const unsigned long long tg0 = __builtin_amdgcn_s_memtime();
#endif
    float distance = gjk_distance(cache, pA, xfA, pB, xfB);
#ifdef NASCAR_PROFILE
    if (prof_cyc) prof_cyc[0] += __builtin_amdgcn_s_memtime() - tg0;
    const unsigned long long ts0 = __builtin_amdgcn_s_memtime();
#endif
    if (distance <= 0.0f) { *state = TOI_OVERLAPPED; out_t = 0.0f; break; }
    if (distance < target + tolerance) { *state = TOI_TOUCHING; out_t = t1; break; }
    SepFn fcn;
    sep_init(fcn, cache, pA, sA, pB, sB, qB, xfA, xfB);
    bool done = false;
    float t2 = tMax;
    // the sweeps' transforms at t2: b2TimeOfImpact re-derives them from t2 for FindMinSeparation; the root
    // finder's last Evaluate was at the same t2 (t2 = t), so its transforms are reused (identical values)
    Xf xfA2 = sweep_xf(sA, t2), xfB2 = sweep_xf_static(sB, t2, qB);
    int pushBackIter = 0;
    for (;;) {
      int indexA, indexB;
      float s2 = sep_find_min(fcn, pA, pB, &indexA, &indexB, xfA2, xfB2);
      if (s2 > target + tolerance) { *state = TOI_SEPARATED; out_t = tMax; done = true; break; }
      if (s2 > target - tolerance) { t1 = t2; xfA = xfA2; xfB = xfB2; break; }
      float s1 = sep_eval(fcn, pA, pB, indexA, indexB, xfA, xfB);   // at t1
      if (s1 < target - tolerance) { *state = TOI_FAILED; out_t = t1; done = true; break; }
      if (s1 <= target + tolerance) { *state = TOI_TOUCHING; out_t = t1; done = true; break; }
      int rootIterCount = 0;
      float a1 = t1, a2 = t2;
      for (;;) {
        float t;
        if (rootIterCount & 1) t = a1 + fdiv_cr((target - s1) * (a2 - a1), s2 - s1);
        else t = 0.5f * (a1 + a2);
        ++rootIterCount;
#ifdef NASCAR_PROFILE
        if (prof_iters) ++prof_iters[1];
#endif
        const Xf xa = sweep_xf(sA, t), xb = sweep_xf_static(sB, t, qB);
        float s = sep_eval(fcn, pA, pB, indexA, indexB, xa, xb);
        if (fabsf(s - target) < tolerance) { t2 = t; xfA2 = xa; xfB2 = xb; break; }
        if (s > target) { a1 = t; s1 = s; } else { a2 = t; s2 = s; }
        if (rootIterCount == 50) break;
      }
      ++pushBackIter;
      if (pushBackIter == 8) break;
    }
    ++iter;
#ifdef NASCAR_PROFILE
    if (prof_iters) ++prof_iters[0];
    if (prof_cyc) prof_cyc[1] += __builtin_amdgcn_s_memtime() - ts0;
#endif
    if (done) break;
    if (iter == 20) { *state = TOI_FAILED; out_t = t1; break; }
  }
#ifdef NASCAR_PROFILE
  if (prof_iters) prof_iters[2] += cache.iters;
#endif
  return out_t;
}

template <int NMAX>
__device__ __forceinline__ void island_solve_toi_buf(Car& c, const LWall* W, const int* cidx, int n, float subdt, float friction,
                                                     VC* vc) {
  BodyState A; A.c = c.c; A.a = c.a; A.v = c.v; A.w = c.w;
  {
  CTIME_BEGIN();
  cs_init<NMAX>(vc, n, c, cidx, W, false, 1.0f);
  CTIME_END(c, 34);   // profile builds: TOI island sub-phases in slots 34-37
  }
  RotCache rcA; rcA.bits = __float_as_uint(c.a) ^ 1u; rcA.q.s = 0.0f; rcA.q.c = 1.0f;   // (empty: no angle matches)
  {
  CTIME_BEGIN();
  int it = 0;
  for (; it < 20; ++it) { if (cs_solve_position<NMAX>(vc, n, A, 1, rcA)) break; }
  CCOUNT(c, 19, it + 1); CCOUNT(c, 18, n);
  CTIME_END(c, 20);
  }
  c.c0 = A.c; c.a0 = A.a;
  {
  CTIME_BEGIN();
  cs_init_velocity<NMAX>(vc, n, c, A);
  CTIME_END(c, 35);
  }
  {
  CTIME_BEGIN();
  SOLVER_ITER_LOOP
  for (int it = 0; it < 6; ++it) cs_solve_velocity<NMAX>(vc, n, A, friction);
  CTIME_END(c, 36);
  }
  CTIME_BEGIN();
  integrate_positions(A, subdt);
  c.c = A.c; c.a = A.a; c.v = A.v; c.w = A.w;
  c.xf.q = rot_cached(rcA, c.a); c.xf.p = vsub(c.c, rmul(c.xf.q, zero2()));   // sync_transform
  report<NMAX>(c, vc, n);
  CTIME_END(c, 37);
}
template <int NMAX>
__device__ __forceinline__ void island_solve_toi_n(Car& c, const LWall* W, const int* cidx, int n, float subdt, float friction) {
  VC vc[NMAX];
  island_solve_toi_buf<NMAX>(c, W, cidx, n, subdt, friction, vc);
}
__device__ inline void island_solve_toi(Car& c, const LWall* W, const int* cidx, int n, float subdt, float friction) {
  if (n <= ISLAND_TWO) island_solve_toi_n<2>(c, W, cidx, n, subdt, friction);
#if ISLAND_MID
  else if (n <= ISLAND_MID) island_solve_toi_n<ISLAND_MID>(c, W, cidx, n, subdt, friction);
#endif
#if ISLAND_LDS   // the general TOI island in the wave's LDS work area, one lane at a time (see solve_island_general)
  else wave_lds_one_at_a_time([&](VC* vc) { island_solve_toi_buf<MAX_ISLAND>(c, W, cidx, n, subdt, friction, vc); });
#else
  else island_solve_toi_n<MAX_ISLAND>(c, W, cidx, n, subdt, friction);
#endif
}

// Exact shortcut for b2TimeOfImpact on a (car, static wall) pair.  The root finder can only report
// TOUCHING -- the one outcome whose alpha differs from 1 -- if the swept car comes within target +
// tolerance (0.005 + 0.00125 m) of the wall: GJK distance(t1) < target + tol, or the separating
// function at t1 (built from the closest features at t1, so >= the distance there) <= target + tol.
// Every car point moves at most |c - c0| + |a - a0| * R_car (R_car = circumradius; the car's centroid is
// its origin) along the sweep, and the separating-axis maximum of the two boxes at the sweep's end pose
// is a lower bound of their distance there.  If that bound minus the motion exceeds target + tol by a
// 1 cm rounding margin, the swept car never comes that close and TOI would return SEPARATED or FAILED:
// alpha = 1 without running it (identical result, verified by every GPU-vs-oracle test).
//
// The bound is a separating-axis one per fixed world axis u (the wall's two axes and the car's two axes at
// the end pose, each oriented from the wall toward the car): the gap along u at sweep parameter beta is
//   gap_u(beta) >= gap_u(end) - max(0, u . (c - c0)) - |a - a0| * R_car
// because u . c(beta) = u . c - (1 - beta) u . (c - c0) (linear sweep) and the rotation moves every car
// point by at most |a - a0| * R_car.  A car sliding along or approaching a wall therefore keeps its end
// pose gap (only motion AWAY from the wall along u widens the interval); distance(beta) >= gap_u(beta).
// Box gaps are exact: gap_u = |u . d| - e_car(u) - e_wall(u) with e(u) = hx |u . x| + hy |u . y|.
// The rounding margin (3 mm) is ~25 ulps of the largest track coordinates (|x| < 1500 m, ulp 1.2e-4).
#define TOI_CULL_DIST (0.005f + 0.00125f + 0.003f)
__device__ __forceinline__ float toi_gap_bound(V2 u, V2 d, V2 dc, V2 cx, V2 cy, V2 wx, V2 wy, float whx, float why) {
  const float s = vdot(u, d);
  const float gap = fabsf(s) - (CAR_HX * fabsf(vdot(u, cx)) + CAR_HY * fabsf(vdot(u, cy)))
                             - (whx * fabsf(vdot(u, wx)) + why * fabsf(vdot(u, wy)));
  const float away = s >= 0.0f ? vdot(u, dc) : -vdot(u, dc);   // motion toward +gap during the sweep
  return gap - fmaxb(0.0f, away);
}
// Second-order rotation bound (round 3), tried when the bound above fails.  Along a fixed axis u (oriented wall ->
// car at the end pose), car vertex k's gap g_k(beta) = u . c(beta) + r cos(a(beta) + psi_k) - (wall terms) is a
// linear function plus a sinusoid of the linear angle a(beta) = a0 + beta (a - a0), so |g_k''| <= r (a - a0)^2 with
// r = R_car, and g_k(beta) >= min(g_k(0), g_k(1)) - r (a - a0)^2 / 8 on [0, 1].  The box gap is the minimum over
// the vertices, hence
//   gap_u(beta) >= min(G_u(start pose), G_u(end pose)) - R_car (a - a0)^2 / 8,
// G_u the separating-axis gap of the two boxes at that pose measured along the end pose's orientation of u.  The
// first-order term |a - a0| R_car above is what keeps a car scraping along a wall (core distance ~15 mm, turning a
// few mrad per step) from being culled; its second-order replacement is ~1e-5 m.  The start pose's rotation is the
// end pose's b2Rot rotated back by a - a0 (Taylor terms to |a - a0|^5, error < 1e-7 for |a - a0| <= 0.1; larger
// rotations are not culled here).
#ifndef TOI_CULL2
#define TOI_CULL2 1
#endif
__device__ __forceinline__ float toi_gap2(V2 u, V2 d1, V2 d0, V2 cx1, V2 cy1, V2 cx0, V2 cy0, float wext) {
  const float s1 = vdot(u, d1), s0 = vdot(u, d0);
  const float g1 = fabsf(s1) - (CAR_HX * fabsf(vdot(u, cx1)) + CAR_HY * fabsf(vdot(u, cy1))) - wext;
  const float g0 = (s1 >= 0.0f ? s0 : -s0) - (CAR_HX * fabsf(vdot(u, cx0)) + CAR_HY * fabsf(vdot(u, cy0))) - wext;
  return fminb(g0, g1);
}
__device__ __forceinline__ bool toi_far_rot2(const Car& c, const LWall& wl, V2 d1, float da, float) {
  if (!(fabsf(da) <= 0.1f)) return false;
  const float R_CAR = 2.80389f;
  const float d2 = da * da;
  const float cd = 1.0f - 0.5f * d2 + d2 * d2 * (1.0f / 24.0f), sd = da * (1.0f - d2 * (1.0f / 6.0f) + d2 * d2 * (1.0f / 120.0f));
  const float qc = c.xf.q.c, qs = c.xf.q.s;
  const float c0c = qc * cd + qs * sd, c0s = qs * cd - qc * sd;   // cos / sin (a - da)
  const V2 cx1 = V(qc, qs), cy1 = V(-qs, qc), cx0 = V(c0c, c0s), cy0 = V(-c0s, c0c);
  const V2 wx = V(wl.qc, wl.qs), wy = V(-wl.qs, wl.qc);
  const V2 d0 = vsub(c.c0, V(wl.px, wl.py));
  // wall extents along its own axes are hx / hy; along the car's axes hx |u . wx| + hy |u . wy|
  float b = toi_gap2(wx, d1, d0, cx1, cy1, cx0, cy0, wl.hx);
  b = fmaxb(b, toi_gap2(wy, d1, d0, cx1, cy1, cx0, cy0, wl.hy));
  b = fmaxb(b, toi_gap2(cx1, d1, d0, cx1, cy1, cx0, cy0, wl.hx * fabsf(vdot(cx1, wx)) + wl.hy * fabsf(vdot(cx1, wy))));
  b = fmaxb(b, toi_gap2(cy1, d1, d0, cx1, cy1, cx0, cy0, wl.hx * fabsf(vdot(cy1, wx)) + wl.hy * fabsf(vdot(cy1, wy))));
  return b - d2 * (R_CAR * 0.125f) > TOI_CULL_DIST;
}
__device__ __forceinline__ bool toi_far(const Car& c, const Poly* pa, const LWall& wl) {
#ifdef NASCAR_NO_TOI_CULL   // A/B and verification builds only
  return false;
#endif
  (void)pa;
  const float R_CAR = 2.80389f;   // > sqrt(CAR_HX^2 + CAR_HY^2) = 2.80323
  const V2 cx = V(c.xf.q.c, c.xf.q.s), cy = V(-c.xf.q.s, c.xf.q.c);
  const V2 wx = V(wl.qc, wl.qs), wy = V(-wl.qs, wl.qc);
  const V2 d = vsub(c.xf.p, V(wl.px, wl.py)), dc = vsub(c.c, c.c0);
  float b = toi_gap_bound(wx, d, dc, cx, cy, wx, wy, wl.hx, wl.hy);
  b = fmaxb(b, toi_gap_bound(wy, d, dc, cx, cy, wx, wy, wl.hx, wl.hy));
  b = fmaxb(b, toi_gap_bound(cx, d, dc, cx, cy, wx, wy, wl.hx, wl.hy));
  b = fmaxb(b, toi_gap_bound(cy, d, dc, cx, cy, wx, wy, wl.hx, wl.hy));
  const float da = c.a - c.a0;
  if (b - fabsf(da) * R_CAR > TOI_CULL_DIST) return true;
#if TOI_CULL2
  return toi_far_rot2(c, wl, d, da, b);
#else
  return false;
#endif
}

// b2World::SolveTOI, wave-cooperative.  Box2D's loop per car: scan the contacts (a cached alpha, or a fresh
// b2TimeOfImpact for each enabled contact without one), take the first contact of minimum alpha, and if
// alpha < 1 advance the body to it, update that contact, solve the TOI island and find new contacts --
// then scan again (the island's contacts lost their cached alphas).  Within one scan a car's sweep is fixed,
// so its fresh TOIs are independent: here every lane first lists the (contact, wall) pairs it needs, the
// wave computes all listed pairs in parallel -- any present lane takes any pair, its owner's sweep read from
// LDS -- and each lane then runs its scan on the results.  The loop runs while any lane of the wave still
// has events, so lanes that are done lend their time to a lane with a long event chain (a car scraping a
// wall re-scans its 2-5 contacts after each event: sequential on one lane before).  Same alphas, same
// scan order, same minimum, so the results are Box2D's.
// b2TimeOfImpact of the car's sweep against static wall wl -> alpha of SolveTOI (1 unless TOUCHING)
__device__ __forceinline__ float toi_alpha(float4 s0, float4 s1, const LWall& wl, int* iters = nullptr,
                                           unsigned long long* cyc = nullptr) {
#ifdef NASCAR_KO_TOIJOBS
  return 1.0f;
#endif
  Poly pa; make_box(&pa, CAR_HX, CAR_HY);
  Poly pb; make_box(&pb, wl.hx, wl.hy);
  Sweep sA; sA.c0 = V(s0.x, s0.y); sA.c = V(s0.z, s0.w); sA.a0 = s1.x; sA.a = s1.y; sA.alpha0 = s1.z;
  Sweep sB; sB.c0 = V(wl.px, wl.py); sB.c = sB.c0; sB.a0 = wl.ang; sB.a = wl.ang; sB.alpha0 = 0.0f;
  int state;
  Rot qw; qw.s = wl.qs; qw.c = wl.qc;
  const float beta = time_of_impact(&state, &pa, sA, &pb, sB, 1.0f, qw, __float_as_uint(wl.ang), iters, cyc);
  return state == TOI_TOUCHING ? fminb(s1.z + (1.0f - s1.z) * beta, 1.0f) : 1.0f;
}
#ifndef TOI_COOP_MANI
#define TOI_COOP_MANI 1
#endif
// contact ci's b2Contact::Update inside a TOI event: from the wave's cooperative manifold when it has one
__device__ __forceinline__ void toi_contact_update(Car& c, int ci, const LWall* W, int moff) {
#if TOI_COOP_MANI
  if (moff + ci < MANI_JOBCAP) { contact_apply(c, ci, W, g_wave_lds[threadIdx.x >> 6].mani.res[moff + ci]); return; }
#endif
  contact_update(c, ci, W);
}
__device__ inline void solve_toi(Car& c, const WallSet& S, float dt, float friction) {
  ToiWaveLDS& L = g_wave_lds[threadIdx.x >> 6].toi;
  const LWall* W = S.W;
  Poly pa; make_box(&pa, CAR_HX, CAR_HY);
  const unsigned long long present = __ballot(1);    // lanes of this wave inside SolveTOI
  const int prank = rank_in(present), npresent = popc64(present);
  const int lane = (int)__lane_id();
  c.alpha0 = 0.0f;
  for (int i = 0; i < c.nct; ++i) { c.ct[i].flags &= ~(CT_TOI | CT_ISLAND); c.ct[i].toiCount = 0; c.ct[i].toi = 1.0f; }
  bool active = true;
  bool had_event = false;   // profile builds' rescan counters only (dead code otherwise)
  for (;;) {
    // (1) this lane's fresh TOIs of this scan: enabled, under the substep cap, no cached alpha, body awake,
    // not provably far (toi_far: alpha = 1 without computing)
    uint32_t need = 0u;   // bit i: contact i needs b2TimeOfImpact
    if (active && c.awake) {
      for (int i = 0; i < c.nct; ++i) {
        DContact& ct = c.ct[i];
        if (!(ct.flags & CT_ENABLED) || ct.toiCount > MAX_SUBSTEPS || (ct.flags & CT_TOI)) continue;
        if (toi_far(c, &pa, ldg(W + ct.wall))) {
          PCOUNT(13, 1); CCOUNT(c, 3, 1);
          if (had_event) CCOUNT(c, 29, 1);   // profile builds: culled in a rescan after this car's event
#ifdef NASCAR_TOI_CULL_CHECK   // check builds: every culled call run anyway; slot 11 counts culled TOUCHING outcomes
          if (toi_alpha(make_float4(c.c0.x, c.c0.y, c.c.x, c.c.y), make_float4(c.a0, c.a, c.alpha0, 0.0f),
                        ldg(W + ct.wall)) < 1.0f) PCOUNT(11, 1);
#endif
          ct.toi = 1.0f; ct.flags |= CT_TOI;
          continue;
        }
        need |= 1u << i;
        if (had_event) CCOUNT(c, 27, 1);   // profile builds: computed in a rescan after this car's event
      }
    }
    // (2) the wave's pairs, numbered lane by lane (prefix over the lanes' counts by bit ballots)
    const int m = __popc(need);
    int off = 0, total = 0;
#pragma unroll
    for (int bit = 0; bit < 5; ++bit) {
      const unsigned long long b = __ballot((m >> bit) & 1);
      off += rank_in(b) << bit;
      total += popc64(b) << bit;
    }
    if (m) { L.sw0[lane] = make_float4(c.c0.x, c.c0.y, c.c.x, c.c.y); L.sw1[lane] = make_float4(c.a0, c.a, c.alpha0, 0.0f); }
    CCOUNT(c, 14, 1);   // profile builds: scans of this wave
#ifdef NASCAR_PROFILE
    const unsigned long long tj0 = __builtin_amdgcn_s_memtime();
#endif
    for (int r0 = 0; r0 < total; r0 += TOI_JOBCAP) {   // wave-uniform
      {
        uint32_t nb = need; int k = off;
        while (nb) {
          const int i = __ffs(nb) - 1; nb &= nb - 1;
          if (k >= r0 && k < r0 + TOI_JOBCAP) L.job[k - r0] = make_int2(lane | (i << 8), c.ct[i].wall);
          ++k;
        }
      }
      wave_lds_sync();
      const int cnt = min(TOI_JOBCAP, total - r0);
      for (int j = prank; j < cnt; j += npresent) {
        const int2 jb = L.job[j];
        const int owner = jb.x & 0xFF;
        PCOUNT(12, 1); CCOUNT(c, 2, 1);
#ifdef NASCAR_PROFILE   // per computing lane: TOI outer / root-finder iterations, GJK and separation-function cycles
        int it2[3] = {0, 0, 0}; unsigned long long cy2[2] = {0ull, 0ull};
        L.res[j] = toi_alpha(L.sw0[owner], L.sw1[owner], ldg(W + jb.y), it2, cy2);
        CCOUNT(c, 6, it2[0]); CCOUNT(c, 7, it2[1]); CCOUNT(c, 9, cy2[0]); CCOUNT(c, 10, cy2[1]);
#else
        L.res[j] = toi_alpha(L.sw0[owner], L.sw1[owner], ldg(W + jb.y));
#endif
#if defined(NASCAR_PROFILE) && defined(NASCAR_TOI_CAPTURE)
        if (g_prof) {
          const unsigned long long k = atomicAdd(&g_prof[TCAP_BASE], 1ull);
          if (k < TCAP_MAX) {
            float4* r = (float4*)&g_prof[TCAP_BASE + 8 + k * 8];
            const LWall w = ldg(W + jb.y);
            r[0] = L.sw0[owner]; r[1] = L.sw1[owner];
            r[2] = make_float4(w.px, w.py, w.qs, w.qc); r[3] = make_float4(w.hx, w.hy, w.ang, __int_as_float(w.key));
          }
        }
#endif
      }
      wave_lds_sync();
      {
        uint32_t nb = need; int k = off;
        while (nb) {
          const int i = __ffs(nb) - 1; nb &= nb - 1;
          if (k >= r0 && k < r0 + TOI_JOBCAP) {
            c.ct[i].toi = L.res[k - r0]; c.ct[i].flags |= CT_TOI;
            if (had_event && c.ct[i].toi < 1.0f) CCOUNT(c, 28, 1);   // profile builds: a rescan's TOUCHING result
          }
          ++k;
        }
      }
      wave_lds_sync();   // the next round's pairs overwrite job / res
    }
#ifdef NASCAR_PROFILE
    CCOUNT(c, 13, __builtin_amdgcn_s_memtime() - tj0);   // the wave's TOI job rounds of this scan
    const unsigned long long te0 = __builtin_amdgcn_s_memtime();
#endif
    // (3) this lane's scan on cached alphas and its event, as Box2D
#ifdef NASCAR_PROFILE
    const unsigned long long ts3 = __builtin_amdgcn_s_memtime();
#endif
    int minC = -1; float minAlpha = 1.0f;
    bool ev = false;
    V2 bc0 = c.c0, bc = c.c; float ba0 = c.a0, ba = c.a, balpha0 = c.alpha0;
    if (active) {
      for (int i = 0; i < c.nct; ++i) {
        const DContact& ct = c.ct[i];
        if (!(ct.flags & CT_ENABLED) || ct.toiCount > MAX_SUBSTEPS || !(ct.flags & CT_TOI)) continue;
        if (ct.toi < minAlpha) { minC = i; minAlpha = ct.toi; }
      }
#ifdef NASCAR_KO_EVENTS
      minC = -1;
#endif
      if (minC < 0 || 1.0f - 10.0f * FLT_EPS < minAlpha) {
        active = false;
      } else {
        ev = true;
        PCOUNT(15, 1); CCOUNT(c, 4, 1);
        had_event = true;
        bc0 = c.c0; bc = c.c; ba0 = c.a0; ba = c.a; balpha0 = c.alpha0;
        {
          float beta = fdiv_cr(minAlpha - c.alpha0, 1.0f - c.alpha0);
          c.c0 = vadd(c.c0, vmul(beta, vsub(c.c, c.c0)));
          c.a0 += beta * (c.a - c.a0);
          c.alpha0 = minAlpha;
          c.c = c.c0; c.a = c.a0;
          sync_transform(c);
        }
      }
    }
    // (3b) wave-cooperative event manifolds: the event's contact update and the island's updates all see the car
    // at its TOI pose (the static walls never move), so b2CollidePolygons of every contact of every event lane is
    // computed up front by any present lane; the owners then apply them in Box2D's order (contact_apply), and
    // only results they reach are used.  Contacts past the LDS job capacity are updated by their owner.
    int moff = MANI_JOBCAP;   // this lane's first result slot (contact i -> slot moff + i)
#ifdef NASCAR_PROFILE
    const unsigned long long tm0 = __builtin_amdgcn_s_memtime();
    if (ev) CCOUNT(c, 38, tm0 - ts3);   // scan on cached alphas + advance to the TOI pose
#endif
#if TOI_COOP_MANI
    if (__ballot(ev)) {   // wave-uniform
      ManiWaveLDS& M = g_wave_lds[threadIdx.x >> 6].mani;
      const int mm = ev ? c.nct : 0;
      int off2 = 0, total2 = 0;
#pragma unroll
      for (int bit = 0; bit < 5; ++bit) {
        const unsigned long long b = __ballot((mm >> bit) & 1);
        off2 += rank_in(b) << bit;
        total2 += popc64(b) << bit;
      }
      if (ev) {
        moff = off2;
        M.xf[lane] = make_float4(c.xf.p.x, c.xf.p.y, c.xf.q.s, c.xf.q.c);
        for (int i = 0; i < c.nct && off2 + i < MANI_JOBCAP; ++i) M.job[off2 + i] = make_int2(lane | (i << 8), c.ct[i].wall);
      }
      wave_lds_sync();
      const int cnt = min(MANI_JOBCAP, total2);
      for (int j = prank; j < cnt; j += npresent) {
        const int2 jb = M.job[j];
        const float4 x = M.xf[jb.x & 0xFF];
        Xf xfA; xfA.p = V(x.x, x.y); xfA.q.s = x.z; xfA.q.c = x.w;
        M.res[j] = contact_manifold(xfA, ldg(W + jb.y));
      }
      wave_lds_sync();
    }
#endif
#ifdef NASCAR_PROFILE
    if (ev) CCOUNT(c, 32, __builtin_amdgcn_s_memtime() - tm0);   // the wave's manifold round for this event
#endif
    if (ev) {
      {
        {
        CTIME_BEGIN();
        toi_contact_update(c, minC, W, moff);
        CTIME_END(c, 12);
        CTIME_END(c, 33);   // (the event contact's own update)
        }
        c.ct[minC].flags &= ~CT_TOI;
        ++c.ct[minC].toiCount;
        if (!(c.ct[minC].flags & CT_ENABLED) || !(c.ct[minC].flags & CT_TOUCH)) {
          c.ct[minC].flags &= ~CT_ENABLED;
          c.c0 = bc0; c.c = bc; c.a0 = ba0; c.a = ba; c.alpha0 = balpha0;
          sync_transform(c);
        } else {
          set_awake(c);
          int cidx[MAX_ISLAND] = {0, 0, 0, 0, 0, 0, 0, 0}; int n = 0;
          island_push(cidx, n, minC); c.ct[minC].flags |= CT_ISLAND;
          {
          CTIME_BEGIN();
          for (int i = 0; i < c.nct; ++i) {
#ifdef NASCAR_KO_EV_CU
            break;
#endif
            if (n == MAX_TOI_CONTACTS) break;
            if (n == MAX_ISLAND) {   // more touching contacts than the island buffer: flag, keep going exactly-as-far-as-possible
              if (!(c.ct[i].flags & CT_ISLAND)) { c.overflow = 2; }
              break;
            }
            if (c.ct[i].flags & CT_ISLAND) continue;
            toi_contact_update(c, i, W, moff);
            if (!(c.ct[i].flags & CT_ENABLED)) continue;
            if (!(c.ct[i].flags & CT_TOUCH)) continue;
            c.ct[i].flags |= CT_ISLAND;
            island_push(cidx, n, i);
          }
          CTIME_END(c, 12);
          }
          float subdt = (1.0f - minAlpha) * dt;
          {
          CTIME_BEGIN();
#ifndef NASCAR_KO_EV_ISLAND
          island_solve_toi(c, W, cidx, n, subdt, friction);
#endif
          CTIME_END(c, 11);
          }
          {
          CTIME_BEGIN();
          sync_fixtures(c);
          for (int i = 0; i < c.nct; ++i) c.ct[i].flags &= ~(CT_TOI | CT_ISLAND);
          CTIME_END(c, 17);
          }
          {
          CTIME_BEGIN();
#ifndef NASCAR_KO_EV_FIND
          find_new_contacts(c, S);
#endif
          CTIME_END(c, 16);
          }
        }
      }
    }
#if TOI_COOP_MANI
    wave_lds_sync();   // every owner's result reads done before the next scan's LDS writes
#endif
#ifdef NASCAR_PROFILE
    CCOUNT(c, 15, __builtin_amdgcn_s_memtime() - te0);   // the wave's event processing of this scan
#endif
    if (!__any(active)) break;   // wave-uniform exit
  }
}

__device__ inline void b2_step(Car& c, const WallSet& S, float dt, float friction) {
  const LWall* W = S.W;
  float inv_dt = dt > 0.0f ? fdiv_cr(1.0f, dt) : 0.0f;
  float dtRatio = c.invdt0 * dt;
#ifdef NASCAR_PROFILE
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  CCOUNT(c, 1, c.nct);
#endif
  // NASCAR_KO_*: knockout builds for timing attribution only (a phase skipped: wrong results, never shipped)
#ifndef NASCAR_KO_COLLIDE
  {
  CTIME_BEGIN();
  collide(c, S);
  CTIME_END(c, 23);
  }
#endif
  PROFB(11);
#ifndef NASCAR_KO_SOLVE
  {
  const bool awake = c.awake != 0;   // b2World::Solve updates the pairs of awake bodies only
  solve(c, S, dt, dtRatio, friction);
#if BP_COOP
  CTIME_BEGIN();
  if (awake && c.moved) CCOUNT(c, 24, 1);
  find_new_contacts_wave(c, S, awake);
  CTIME_END(c, 21);
#endif
  }
#endif
  PROFB(13);
#ifdef NASCAR_PROFILE
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
#endif
#ifndef NASCAR_KO_TOI
#if MODEL_PRIO == 2   // A/B: waves in SolveTOI issue ahead of co-resident waves
  __builtin_amdgcn_s_setprio(3);
#endif
  solve_toi(c, S, dt, friction);
#if MODEL_PRIO == 2
  __builtin_amdgcn_s_setprio(0);
#endif
#endif
#ifdef NASCAR_PROFILE
  const unsigned long long t2 = __builtin_amdgcn_s_memtime();
  CCOUNT(c, 0, t2 - t0); (void)t1;
#endif
  c.invdt0 = inv_dt;
  c.force = zero2(); c.torque = 0.0f;
}

// b2Body::SetTransform
__device__ inline void set_transform(Car& c, const WallSet& S, V2 pos, float angle) {
  c.xf.q = rot_set(angle);
  c.xf.p = pos;
  c.c = xmul(c.xf, zero2()); c.a = angle;
  c.c0 = c.c; c.a0 = angle;
  move_proxy(c, c.xf, c.xf);
  find_new_contacts(c, S);
}

}  // namespace nascar
