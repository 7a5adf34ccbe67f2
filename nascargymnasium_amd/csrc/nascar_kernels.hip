// nascar_kernels.hip -- fused batched CarEnv step for MI355X (gfx950) + the C ABI.
//
// Execution model: one workgroup = floor(256 / C) whole envs of ONE track
// (C cars each, one lane per car).  The track's ~730 wall boxes are staged once
// per workgroup into LDS and shared by the Box2D broadphase/narrowphase, the 16
// distance-sensor rays of every car and the on-track query.  Env-level coupling
// (lap-reset pending, termination, auto-reset) is reduced through LDS between
// phases separated by __syncthreads().  All per-car state lives in HBM as SoA
// (nascar_layout.h) and is read/written once per step.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <thread>
#include <cmath>
#include <string>
#include <memory>
#include <mutex>
#include <unordered_map>
#include <deque>
#include <fcntl.h>
#include <sys/file.h>
#include <sys/stat.h>
#include <unistd.h>
#include <vector>

#include "../../include/nascar.h"
#include "nascar_device.h"
#include "nascar_actor.h"
#include "nascar_rays.h"

#pragma clang fp contract(off)

using namespace nascar;

#define MAX_SEG 64

#ifdef NASCAR_DEBUG
__device__ double* g_dbg = nullptr;   // debug build only: intermediate taps of one car
__device__ int g_dbg_car = -1;
#define DBG(n, slot, val) do { if ((n) == g_dbg_car && g_dbg) g_dbg[slot] = (double)(val); } while (0)
#else
#define DBG(n, slot, val) do { } while (0)
#endif


// ------------------------------------------------------------------ device-side tables
struct DSeg {   // per segment, float64 (src/track_generator.py TrackSegment)
  double sx, sy, ex, ey, width, banking, la, chord;  // la: banking lateral assist (src/car.py:527-533)
};
// Ray-candidate lists ("beams"), built on the host (build_beams): for every cell (nascar_set_beam_cell) near the
// walls and every one of BEAM_NB direction bins, the walls that a ray starting anywhere in the cell with a
// direction in the bin can reach within 250 m, sorted by a lower bound of their distance from the cell.
// Entry (16 bits) = bound code << wbits | wall index (wbits = 10 up to 1024 walls, up to 13 for 8192): code c stands
// for the bound c^2 * kq m, rounded down from the wall's exact bound (c < cmax = 2^(16 - wbits) - 1, the sentinel's
// code, past every hit), so the codes are conservative and ascend along a list.  A ray walks its list and stops at the first entry whose bound exceeds its best hit so far: the minimum exact
// fraction over the walls visited is the minimum over all walls, i.e. the reference's Box2D RayCast result.
#ifndef BEAM_NB
#define BEAM_NB 256       // direction bins (measured 64: 44.2 us, 128: 41.7, 256: 38.7, 512: 39.1) (a multiple of 16: ray i is BEAM_NB / 16 bins from ray i + 1)
#endif
#define BEAM_STRIDE (BEAM_NB / 16)
// list slot of a bin: the 16 bins of one residue mod BEAM_STRIDE are adjacent, so a car's 16 rays read
// 16 adjacent lists
__host__ __device__ __forceinline__ int beam_slot(int bin) { return (bin % BEAM_STRIDE) * 16 + bin / BEAM_STRIDE; }
__host__ __device__ __forceinline__ int beam_bin(int slot) { return (slot % 16) * BEAM_STRIDE + slot / 16; }
#define BEAM_MAX_WALL_BITS 13                  // tracks with more than 8192 walls get no lists (the wall-group walk)
#define BEAM_PAD 0xFFFFu                       // sentinel: the largest code, stops every walk
#define BEAM_CONT_MAX 0xFFFFu                  // continuation entries of one cell (16-bit offsets from the cell's base)
struct BeamGrid {
  float ox, oy, inv_cell; int nx, ny;
  uint32_t wbits, wmask, cmax; float kq;   // entry layout: wall index bits, their mask, sentinel code, bound scale (m)
  // the cell map in chunks of BEAM_CHUNK cells along x, [ny][nxc]: (first list of the chunk's first built cell = its
  // id * BEAM_NB, the chunk's first ent[] index, the mask of its built cells, 0) -- the built cells of a chunk have
  // consecutive ids, so a cell's list base is the chunk's plus BEAM_NB per built cell below it.  ~0.5 MB per track
  // (a dense int2 per cell was ~9 MB, a random 128-byte line per car that no L2 held; this table stays cached)
  const int4* chunk; int nxc;
  const uint16_t* ent;      // list continuations, each closed by a BEAM_PAD sentinel
  // [built cells * BEAM_NB] 8-byte head records: the first BEAM_HEAD entries of each list (padded with BEAM_PAD) and
  // the offset + 1 of the list's continuation from its chunk's first ent[] index (0: none), so a walk starts with one
  // 8-byte load and reads the rest in chunks of RAY_CHUNK entries up to the sentinel.  (Round 5's 16-byte heads held
  // three 32-bit entries and an absolute index: 256 B of heads per car and step against 128.)
  const uint2* head;
};
#define BEAM_HEAD 3
#ifndef RAY_CHUNK
#define RAY_CHUNK 4    // list entries past the head requested together
#endif
// an entry's distance bound in m (the sentinel's: beyond every hit) and its wall
__device__ __forceinline__ float beam_bound(const BeamGrid& G, uint32_t v) {
  const uint32_t c = v >> G.wbits;
  return c >= G.cmax ? 1e30f : (float)(c * c) * G.kq;
}
__device__ __forceinline__ int beam_wall(const BeamGrid& G, uint32_t v) { return (int)(v & G.wmask); }
// a walk goes on past an entry while its bound is within the best hit (fraction bi of the 250 m ray), with margin
__device__ __forceinline__ bool beam_beyond(const BeamGrid& G, uint32_t v, float bi) {
  return beam_bound(G, v) > bi * 250.0f * 1.00001f + 0.01f;
}
#define BEAM_CHUNK 32
struct BeamHead { uint2 w; uint32_t cb; };   // the head record and its chunk's first ent[] index
__device__ __forceinline__ BeamHead beam_head(const BeamGrid& G, int2 cell, int li) {
  BeamHead h;
  h.w = ldg(G.head + li);
  h.cb = (uint32_t)cell.y;
  return h;
}
#define LDS_PER_CU ((size_t)160 * 1024)   // gfx950: 160 KiB of LDS per CU, all of which one workgroup may declare
struct TrackDev {
  LWall* walls; int nwall;
  const float4* wfat;  // [nwall] broadphase fat AABBs
  DSeg* segs; int nseg;
  double* prefix;      // cumulative chord length before segment k (src/car_env.py:1593-1600)
  double total_length; int startline; int has_banking;
  WallGrid bp, sn;
  const float4* groups; int ngroup;   // sensor wall groups: (cx, cy, radius incl. margin, first | count << 16)
  const float4* swall;                // [2 * nwall] sensor image: (px, py, rad + 0.25, hx), (qs, qc, hy, 0)
  BeamGrid beam;                      // per (cell, direction bin) candidate walls of one ray (ray_sensor_kernel)
};

struct Params {
  int E, C, N, epb, nblocks, reset_on_lap;
  float dt_f; double dt_d; float friction;
  double start_x, start_y; float start_angle;
  float* f32; double* f64; int* i32; double* acc;
  DContact* ct; int* act_key; float* act_n;
  double* env_time; int* env_i32;
  const int* blk_track; const int* blk_env;
  const TrackDev* tracks;
  float4* pose;        // [2][N] sensor hand-off: (x, y, angle, mode) -- see sensor_kernel
  // [E] this step's auto-reset envs (the logic writes every env's byte): the step's sensor passes read an env's pass-B
  // pose only when its byte is set, so the pass-B records of the other cars are neither cleared nor read every step
  uint8_t* reset_env;
  double2* pose_cs;    // [2][N] cos, sin of (double)angle for the ray end points (computed once per car)
  const double2* ray_cs;   // [16] cos, sin of the ray offsets radians(22.5 i) (nascar_rays.h)
  double* ctl;         // [N][4] rule-driver state of the device action sources (policy_car)
  float* vhist;        // [VH_RING][N] speed history for validate_performance, or null (nascar_set_perf_history)
  int car_contact;     // build-only extension (nascar_set_car_contact): car-car contact inside each env; 0 = reference
  // block map shortcuts (prepare()): map_identity = blk_env[s] is s (< E) or -1, one_track >= 0 = every
  // block's track; they spare each kernel's first dependent load
  int map_identity, one_track;
  int blk0;            // first step-kernel workgroup of this launch (sharded rollout, nascar_set_rollout_streams); else 0
};
__device__ __forceinline__ int blk_env_of(const Params& P, int el, int s) {
  if (el >= P.epb) return -1;
  if (P.map_identity) return s < P.E ? s : -1;
  return P.blk_env[s];
}
__device__ __forceinline__ int blk_track_of(const Params& P, int b) { return P.one_track >= 0 ? P.one_track : P.blk_track[b]; }
// a workgroup of no track: the device-built block map's workgroups past the last track's (random-track mode); every
// kernel returns first for them (never taken with the host-built map, whose workgroups all hold envs)
#ifndef EMPTY_GUARD
#define EMPTY_GUARD 1
#endif
__device__ __forceinline__ bool blk_empty(const Params& P, int b) { return EMPTY_GUARD && P.one_track < 0 && P.blk_track[b] < 0; }
// The step kernels' workgroup (block-map index) of this dispatch slot.  The dispatcher deals a launch's workgroups
// round-robin over the 8 XCDs (slot b on XCD b % 8), each with its own L2; with XCD_REMAP, each XCD takes a contiguous
// run of the launch's workgroups instead, so the state cache lines two neighbouring workgroups share (a workgroup's
// SoA run of cars rarely ends on a 128-B line) are fetched into one L2, not two.
#ifndef XCD_REMAP
#define XCD_REMAP 1
#endif
__device__ __forceinline__ int wg_block(const Params& P) {
#if XCD_REMAP
  const int nb = gridDim.x, b = blockIdx.x, q = nb >> 3, r = nb & 7, x = b & 7;
  return P.blk0 + x * q + min(x, r) + (b >> 3);
#else
  return blockIdx.x + P.blk0;
#endif
}
// BeamGrid record of the cell holding (x, y): (list base = built cell id * BEAM_NB, its chunk's first ent[] index);
// list base -1 outside the built cells
__device__ __forceinline__ int2 beam_cell(const BeamGrid& G, float x, float y) {
  const float fx = (x - G.ox) * G.inv_cell, fy = (y - G.oy) * G.inv_cell;
  if (!(fx >= 0.0f && fy >= 0.0f && fx < (float)G.nx && fy < (float)G.ny)) return make_int2(-1, 0);
  const int cx = (int)fx;
  const int4 ch = ldg(G.chunk + (int)fy * G.nxc + cx / BEAM_CHUNK);
  const uint32_t bit = 1u << (cx % BEAM_CHUNK), m = (uint32_t)ch.z;
  if (!(m & bit)) return make_int2(-1, 0);
  return make_int2(ch.x + __popc(m & (bit - 1u)) * BEAM_NB, ch.y);
}

#define F32P(P, f) ((P).f32 + (size_t)F32_##f * (P).N)
#define F64P(P, f) ((P).f64 + (size_t)F64_##f * (P).N)
#define I32P(P, f) ((P).i32 + (size_t)I32_##f * (P).N)

// ------------------------------------------------------------------ load / store of one car
__device__ inline void car_load(const Params& P, int n, Car& c) {
  c.c = V(F32P(P, cx)[n], F32P(P, cy)[n]); c.a = F32P(P, a)[n];
  c.v = V(F32P(P, vx)[n], F32P(P, vy)[n]); c.w = F32P(P, w)[n];
  c.xf.q.s = F32P(P, qs)[n]; c.xf.q.c = F32P(P, qc)[n]; c.xf.p = V(F32P(P, xpx)[n], F32P(P, xpy)[n]);
  c.sleep = F32P(P, sleep)[n]; c.invdt0 = F32P(P, invdt0)[n];
  c.fat.lo = V(F32P(P, flox)[n], F32P(P, floy)[n]); c.fat.hi = V(F32P(P, fhix)[n], F32P(P, fhiy)[n]);
  c.cum_reward = F32P(P, cum_reward)[n]; c.cum_reward_info = F32P(P, cum_reward_info)[n];
  c.rpm = F64P(P, rpm)[n]; c.pvx = F64P(P, pvx)[n]; c.pvy = F64P(P, pvy)[n];
  c.lfm = F64P(P, lfm)[n]; c.slip = F64P(P, slip)[n]; c.bank = F64P(P, bank)[n];
  c.load[0] = F64P(P, load0)[n]; c.load[1] = F64P(P, load1)[n]; c.load[2] = F64P(P, load2)[n]; c.load[3] = F64P(P, load3)[n];
  c.temp[0] = F64P(P, temp0)[n]; c.temp[1] = F64P(P, temp1)[n]; c.temp[2] = F64P(P, temp2)[n]; c.temp[3] = F64P(P, temp3)[n];
  c.wear[0] = F64P(P, wear0)[n]; c.wear[1] = F64P(P, wear1)[n]; c.wear[2] = F64P(P, wear2)[n]; c.wear[3] = F64P(P, wear3)[n];
  c.imp = F64P(P, imp)[n];
  c.lt_start = F64P(P, lt_start)[n]; c.lt_cur = F64P(P, lt_cur)[n]; c.lt_last = F64P(P, lt_last)[n];
  c.lt_best = F64P(P, lt_best)[n]; c.lt_px = F64P(P, lt_px)[n]; c.lt_py = F64P(P, lt_py)[n]; c.lt_dist = F64P(P, lt_dist)[n];
  c.cum_impact = F64P(P, cum_impact)[n]; c.stuck_dur = F64P(P, stuck_dur)[n];
  c.stuck_sx = F64P(P, stuck_sx)[n]; c.stuck_sy = F64P(P, stuck_sy)[n];
  c.prev_px = F64P(P, prev_px)[n]; c.prev_py = F64P(P, prev_py)[n];
  c.prog_hist = F64P(P, prog_hist)[n]; c.back = F64P(P, back)[n]; c.prev_back = F64P(P, prev_back)[n];
  c.imp_at_obs = F64P(P, imp_at_obs)[n];
  c.awake = I32P(P, awake)[n]; c.nct = I32P(P, nct)[n]; c.overflow = I32P(P, overflow)[n];
  c.acc_len = I32P(P, acc_len)[n]; c.acc_head = I32P(P, acc_head)[n];
  c.imp_present = I32P(P, imp_present)[n]; c.nact = I32P(P, nact)[n];
  c.lt_timing = I32P(P, lt_timing)[n]; c.lt_has_last = I32P(P, lt_has_last)[n]; c.lt_has_best = I32P(P, lt_has_best)[n];
  c.lt_crossed = I32P(P, lt_crossed)[n]; c.lt_has_pos = I32P(P, lt_has_pos)[n]; c.lt_laps = I32P(P, lt_laps)[n];
  c.disabled = I32P(P, disabled)[n]; c.has_stuck_start = I32P(P, has_stuck_start)[n];
  c.first_step = I32P(P, first_step)[n]; c.prev_laps = I32P(P, prev_laps)[n];
  c.just_disabled = 0;
  c.force = zero2(); c.torque = 0.0f; c.c0 = c.c; c.a0 = c.a; c.alpha0 = 0.0f; c.moved = 0;
  c.ct = P.ct + (size_t)n * MAXC; c.act_key = P.act_key + (size_t)n * MAXC; c.act_n = P.act_n + (size_t)n * MAXC * 2;
  c.acc = nullptr;
}
__device__ inline void car_store(const Params& P, int n, const Car& c) {
  F32P(P, cx)[n] = c.c.x; F32P(P, cy)[n] = c.c.y; F32P(P, a)[n] = c.a;
  F32P(P, vx)[n] = c.v.x; F32P(P, vy)[n] = c.v.y; F32P(P, w)[n] = c.w;
  F32P(P, qs)[n] = c.xf.q.s; F32P(P, qc)[n] = c.xf.q.c; F32P(P, xpx)[n] = c.xf.p.x; F32P(P, xpy)[n] = c.xf.p.y;
  F32P(P, sleep)[n] = c.sleep; F32P(P, invdt0)[n] = c.invdt0;
  F32P(P, flox)[n] = c.fat.lo.x; F32P(P, floy)[n] = c.fat.lo.y; F32P(P, fhix)[n] = c.fat.hi.x; F32P(P, fhiy)[n] = c.fat.hi.y;
  F32P(P, cum_reward)[n] = c.cum_reward; F32P(P, cum_reward_info)[n] = c.cum_reward_info;
  F64P(P, rpm)[n] = c.rpm; F64P(P, pvx)[n] = c.pvx; F64P(P, pvy)[n] = c.pvy;
  F64P(P, lfm)[n] = c.lfm; F64P(P, slip)[n] = c.slip; F64P(P, bank)[n] = c.bank;
  F64P(P, load0)[n] = c.load[0]; F64P(P, load1)[n] = c.load[1]; F64P(P, load2)[n] = c.load[2]; F64P(P, load3)[n] = c.load[3];
  F64P(P, temp0)[n] = c.temp[0]; F64P(P, temp1)[n] = c.temp[1]; F64P(P, temp2)[n] = c.temp[2]; F64P(P, temp3)[n] = c.temp[3];
  F64P(P, wear0)[n] = c.wear[0]; F64P(P, wear1)[n] = c.wear[1]; F64P(P, wear2)[n] = c.wear[2]; F64P(P, wear3)[n] = c.wear[3];
  F64P(P, imp)[n] = c.imp;
  F64P(P, lt_start)[n] = c.lt_start; F64P(P, lt_cur)[n] = c.lt_cur; F64P(P, lt_last)[n] = c.lt_last;
  F64P(P, lt_best)[n] = c.lt_best; F64P(P, lt_px)[n] = c.lt_px; F64P(P, lt_py)[n] = c.lt_py; F64P(P, lt_dist)[n] = c.lt_dist;
  F64P(P, cum_impact)[n] = c.cum_impact; F64P(P, stuck_dur)[n] = c.stuck_dur;
  F64P(P, stuck_sx)[n] = c.stuck_sx; F64P(P, stuck_sy)[n] = c.stuck_sy;
  F64P(P, prev_px)[n] = c.prev_px; F64P(P, prev_py)[n] = c.prev_py;
  F64P(P, prog_hist)[n] = c.prog_hist; F64P(P, back)[n] = c.back; F64P(P, prev_back)[n] = c.prev_back;
  F64P(P, imp_at_obs)[n] = c.imp_at_obs;
  I32P(P, awake)[n] = c.awake; I32P(P, nct)[n] = c.nct; I32P(P, overflow)[n] = c.overflow;
  I32P(P, acc_len)[n] = c.acc_len; I32P(P, acc_head)[n] = c.acc_head;
  I32P(P, imp_present)[n] = c.imp_present; I32P(P, nact)[n] = c.nact;
  I32P(P, lt_timing)[n] = c.lt_timing; I32P(P, lt_has_last)[n] = c.lt_has_last; I32P(P, lt_has_best)[n] = c.lt_has_best;
  I32P(P, lt_crossed)[n] = c.lt_crossed; I32P(P, lt_has_pos)[n] = c.lt_has_pos; I32P(P, lt_laps)[n] = c.lt_laps;
  I32P(P, disabled)[n] = c.disabled; I32P(P, has_stuck_start)[n] = c.has_stuck_start;
  I32P(P, first_step)[n] = c.first_step; I32P(P, prev_laps)[n] = c.prev_laps;
}

// Staged load/store for model_kernel: only the body, vehicle-model and listener fields are
// live through update_physics + the Box2D step; the model fields are written back right
// after update_physics (a compiler memory barrier stops the reload being forwarded) and the
// lap-timer / bookkeeping fields are loaded after the Box2D step.  Register pressure, not
// traffic, is what this buys (the re-read hits L2).
__device__ inline void car_load_phys(const Params& P, int n, Car& c) {
  c.c = V(F32P(P, cx)[n], F32P(P, cy)[n]); c.a = F32P(P, a)[n];
  c.v = V(F32P(P, vx)[n], F32P(P, vy)[n]); c.w = F32P(P, w)[n];
  c.xf.q.s = F32P(P, qs)[n]; c.xf.q.c = F32P(P, qc)[n]; c.xf.p = V(F32P(P, xpx)[n], F32P(P, xpy)[n]);
  c.sleep = F32P(P, sleep)[n]; c.invdt0 = F32P(P, invdt0)[n];
  c.fat.lo = V(F32P(P, flox)[n], F32P(P, floy)[n]); c.fat.hi = V(F32P(P, fhix)[n], F32P(P, fhiy)[n]);
  c.rpm = F64P(P, rpm)[n]; c.pvx = F64P(P, pvx)[n]; c.pvy = F64P(P, pvy)[n];
  c.lfm = F64P(P, lfm)[n]; c.slip = F64P(P, slip)[n]; c.bank = F64P(P, bank)[n];
  c.load[0] = F64P(P, load0)[n]; c.load[1] = F64P(P, load1)[n]; c.load[2] = F64P(P, load2)[n]; c.load[3] = F64P(P, load3)[n];
  c.temp[0] = F64P(P, temp0)[n]; c.temp[1] = F64P(P, temp1)[n]; c.temp[2] = F64P(P, temp2)[n]; c.temp[3] = F64P(P, temp3)[n];
  c.wear[0] = F64P(P, wear0)[n]; c.wear[1] = F64P(P, wear1)[n]; c.wear[2] = F64P(P, wear2)[n]; c.wear[3] = F64P(P, wear3)[n];
  c.imp = F64P(P, imp)[n];
  c.awake = I32P(P, awake)[n]; c.nct = I32P(P, nct)[n]; c.overflow = I32P(P, overflow)[n];
  c.acc_len = I32P(P, acc_len)[n]; c.acc_head = I32P(P, acc_head)[n];
  c.imp_present = I32P(P, imp_present)[n]; c.nact = I32P(P, nact)[n];
  c.disabled = I32P(P, disabled)[n];
  c.just_disabled = 0;
  c.force = zero2(); c.torque = 0.0f; c.c0 = c.c; c.a0 = c.a; c.alpha0 = 0.0f; c.moved = 0;
  c.ct = P.ct + (size_t)n * MAXC; c.act_key = P.act_key + (size_t)n * MAXC; c.act_n = P.act_n + (size_t)n * MAXC * 2;
  c.acc = nullptr;
}
__device__ inline void car_store_model(const Params& P, int n, const Car& c) {
  F64P(P, rpm)[n] = c.rpm; F64P(P, pvx)[n] = c.pvx; F64P(P, pvy)[n] = c.pvy;
  F64P(P, lfm)[n] = c.lfm; F64P(P, slip)[n] = c.slip;
  F64P(P, load0)[n] = c.load[0]; F64P(P, load1)[n] = c.load[1]; F64P(P, load2)[n] = c.load[2]; F64P(P, load3)[n] = c.load[3];
  F64P(P, temp0)[n] = c.temp[0]; F64P(P, temp1)[n] = c.temp[1]; F64P(P, temp2)[n] = c.temp[2]; F64P(P, temp3)[n] = c.temp[3];
  F64P(P, wear0)[n] = c.wear[0]; F64P(P, wear1)[n] = c.wear[1]; F64P(P, wear2)[n] = c.wear[2]; F64P(P, wear3)[n] = c.wear[3];
  I32P(P, acc_len)[n] = c.acc_len; I32P(P, acc_head)[n] = c.acc_head;
}
__device__ inline void car_reload_tyres(const Params& P, int n, Car& c) {
  c.load[0] = F64P(P, load0)[n]; c.load[1] = F64P(P, load1)[n]; c.load[2] = F64P(P, load2)[n]; c.load[3] = F64P(P, load3)[n];
  c.temp[0] = F64P(P, temp0)[n]; c.temp[1] = F64P(P, temp1)[n]; c.temp[2] = F64P(P, temp2)[n]; c.temp[3] = F64P(P, temp3)[n];
  c.wear[0] = F64P(P, wear0)[n]; c.wear[1] = F64P(P, wear1)[n]; c.wear[2] = F64P(P, wear2)[n]; c.wear[3] = F64P(P, wear3)[n];
}
__device__ inline void car_load_logic(const Params& P, int n, Car& c) {
  c.cum_reward = F32P(P, cum_reward)[n]; c.cum_reward_info = F32P(P, cum_reward_info)[n];
  c.lt_start = F64P(P, lt_start)[n]; c.lt_cur = F64P(P, lt_cur)[n]; c.lt_last = F64P(P, lt_last)[n];
  c.lt_best = F64P(P, lt_best)[n]; c.lt_px = F64P(P, lt_px)[n]; c.lt_py = F64P(P, lt_py)[n]; c.lt_dist = F64P(P, lt_dist)[n];
  c.cum_impact = F64P(P, cum_impact)[n]; c.stuck_dur = F64P(P, stuck_dur)[n];
  c.stuck_sx = F64P(P, stuck_sx)[n]; c.stuck_sy = F64P(P, stuck_sy)[n];
  c.prev_px = F64P(P, prev_px)[n]; c.prev_py = F64P(P, prev_py)[n];
  c.prog_hist = F64P(P, prog_hist)[n]; c.back = F64P(P, back)[n]; c.prev_back = F64P(P, prev_back)[n];
  c.imp_at_obs = F64P(P, imp_at_obs)[n];
  c.lt_timing = I32P(P, lt_timing)[n]; c.lt_has_last = I32P(P, lt_has_last)[n]; c.lt_has_best = I32P(P, lt_has_best)[n];
  c.lt_crossed = I32P(P, lt_crossed)[n]; c.lt_has_pos = I32P(P, lt_has_pos)[n]; c.lt_laps = I32P(P, lt_laps)[n];
  c.has_stuck_start = I32P(P, has_stuck_start)[n];
  c.first_step = I32P(P, first_step)[n]; c.prev_laps = I32P(P, prev_laps)[n];
}

// model_kernel -> logic_kernel hand-off: the body / listener fields the Box2D step produced
__device__ inline void car_store_body(const Params& P, int n, const Car& c) {
  F32P(P, cx)[n] = c.c.x; F32P(P, cy)[n] = c.c.y; F32P(P, a)[n] = c.a;
  F32P(P, vx)[n] = c.v.x; F32P(P, vy)[n] = c.v.y; F32P(P, w)[n] = c.w;
  F32P(P, qs)[n] = c.xf.q.s; F32P(P, qc)[n] = c.xf.q.c; F32P(P, xpx)[n] = c.xf.p.x; F32P(P, xpy)[n] = c.xf.p.y;
  F32P(P, sleep)[n] = c.sleep; F32P(P, invdt0)[n] = c.invdt0;
  F32P(P, flox)[n] = c.fat.lo.x; F32P(P, floy)[n] = c.fat.lo.y; F32P(P, fhix)[n] = c.fat.hi.x; F32P(P, fhiy)[n] = c.fat.hi.y;
  F64P(P, imp)[n] = c.imp;
  I32P(P, awake)[n] = c.awake; I32P(P, nct)[n] = c.nct; I32P(P, overflow)[n] = c.overflow;
  I32P(P, imp_present)[n] = c.imp_present; I32P(P, nact)[n] = c.nact;
}
__device__ inline void car_load_body(const Params& P, int n, Car& c) {
  c.c = V(F32P(P, cx)[n], F32P(P, cy)[n]); c.a = F32P(P, a)[n];
  c.v = V(F32P(P, vx)[n], F32P(P, vy)[n]); c.w = F32P(P, w)[n];
  c.xf.q.s = F32P(P, qs)[n]; c.xf.q.c = F32P(P, qc)[n]; c.xf.p = V(F32P(P, xpx)[n], F32P(P, xpy)[n]);
  c.sleep = F32P(P, sleep)[n]; c.invdt0 = F32P(P, invdt0)[n];
  c.fat.lo = V(F32P(P, flox)[n], F32P(P, floy)[n]); c.fat.hi = V(F32P(P, fhix)[n], F32P(P, fhiy)[n]);
  c.imp = F64P(P, imp)[n];
  c.awake = I32P(P, awake)[n]; c.nct = I32P(P, nct)[n]; c.overflow = I32P(P, overflow)[n];
  c.imp_present = I32P(P, imp_present)[n]; c.nact = I32P(P, nact)[n];
  c.disabled = I32P(P, disabled)[n];
  c.just_disabled = 0;
  c.force = zero2(); c.torque = 0.0f; c.c0 = c.c; c.a0 = c.a; c.alpha0 = 0.0f; c.moved = 0;
  c.ct = P.ct + (size_t)n * MAXC; c.act_key = P.act_key + (size_t)n * MAXC; c.act_n = P.act_n + (size_t)n * MAXC * 2;
  c.acc = nullptr;
}
// logic_kernel's write-back: every field but the vehicle-model ones (car_store_model) and the body
// ones only the model kernel changes
__device__ inline void car_store_logic(const Params& P, int n, const Car& c) {
  F32P(P, cum_reward)[n] = c.cum_reward; F32P(P, cum_reward_info)[n] = c.cum_reward_info;
  F64P(P, bank)[n] = c.bank; F64P(P, imp)[n] = c.imp;
  F64P(P, lt_start)[n] = c.lt_start; F64P(P, lt_cur)[n] = c.lt_cur; F64P(P, lt_last)[n] = c.lt_last;
  F64P(P, lt_best)[n] = c.lt_best; F64P(P, lt_px)[n] = c.lt_px; F64P(P, lt_py)[n] = c.lt_py; F64P(P, lt_dist)[n] = c.lt_dist;
  F64P(P, cum_impact)[n] = c.cum_impact; F64P(P, stuck_dur)[n] = c.stuck_dur;
  F64P(P, stuck_sx)[n] = c.stuck_sx; F64P(P, stuck_sy)[n] = c.stuck_sy;
  F64P(P, prev_px)[n] = c.prev_px; F64P(P, prev_py)[n] = c.prev_py;
  F64P(P, prog_hist)[n] = c.prog_hist; F64P(P, back)[n] = c.back; F64P(P, prev_back)[n] = c.prev_back;
  F64P(P, imp_at_obs)[n] = c.imp_at_obs;
  I32P(P, imp_present)[n] = c.imp_present;
  I32P(P, lt_timing)[n] = c.lt_timing; I32P(P, lt_has_last)[n] = c.lt_has_last; I32P(P, lt_has_best)[n] = c.lt_has_best;
  I32P(P, lt_crossed)[n] = c.lt_crossed; I32P(P, lt_has_pos)[n] = c.lt_has_pos; I32P(P, lt_laps)[n] = c.lt_laps;
  I32P(P, disabled)[n] = c.disabled; I32P(P, has_stuck_start)[n] = c.has_stuck_start;
  I32P(P, first_step)[n] = c.first_step; I32P(P, prev_laps)[n] = c.prev_laps;
}

// ------------------------------------------------------------------ tyres (src/tyre.py, src/tyre_manager.py)
__device__ inline double tyre_grip(double T, double wear) {
  double tg;
  if (85.0 <= T && T <= 105.0) tg = 1.5;
  else {
    double dev = T < 85.0 ? 85.0 - T : T - 105.0;
    double g = 1.5 - dev * 0.02;
    tg = pymax(0.8, g);
  }
  double wf = 1.0 - (wear / 100.0) * (1.0 - 0.5);
  return tg * wf;
}
__device__ inline double total_grip(const Car& c) {
  double tg = 0.0, tw = 0.0;
#pragma unroll
  for (int i = 0; i < 4; ++i) { tg += tyre_grip(c.temp[i], c.wear[i]) * c.load[i]; tw += c.load[i]; }
  return tw > 0 ? tg / tw : 0.0;
}
__device__ inline void tyre_update(Car& c, int i, double dt, double load, double ff, double speed, double lat, double slip) {
  c.load[i] = load;
  double ns = pymin(speed / CAR_MAX_SPEED_MS, 2.0);
  double sf = 1.0 + P2(ns);
  double fp = fabs(ff) * 0.040 * sf;
  double ah = 0.0;
  if (speed > 50.0) ah = P2(speed) * 0.0002;
  double th = (fp + ah) * dt / 125.0;
  double td = c.temp[i] - 25.0;
  double ce = 0.01;
  if (speed > 50.0) { double cr = pymin(0.8, speed / 100.0); ce *= (1.0 - cr * 0.5); }
  double cool = td * ce;
  double tdec = cool * dt;
  c.temp[i] += th - tdec;
  c.temp[i] = pymax(25.0, pymin(120.0, c.temp[i]));
  double T = c.temp[i];
  double fwr = fabs(ff) * 0.00001;
  double tm;
  if (85.0 <= T && T <= 105.0) tm = 1.0;
  else if (T > 105.0) tm = 1.0 + ((T - 105.0) / 20.0);
  else tm = 1.0 + ((85.0 - T) / 30.0);
  double lf = load / STATIC_LOAD_PER_TYRE;
  double lm = pymax(0.5, lf);
  double wf = pymax(1.0, T / 80.0);
  double skmh = speed * 3.6;
  double swf = 1.0 + (skmh / 400.0) * 3.0;
  swf = pymin(swf, 3.0);
  double lat_g = fabs(lat) / 9.81;
  double cwf;
  if (lat_g > 2.0) { double ex = lat_g - 2.0; cwf = 1.0 + (ex * 1.5); cwf = pymin(cwf, 2.5); }
  else cwf = 1.0;
  double slwf = 1.0 + (fabs(slip) / 45.0) * (3.0 - 1.0);
  slwf = pymin(slwf, 3.0);
  double tot = tm * lm * wf * swf * cwf * slwf;
  double rate = fwr * tot;
  c.wear[i] += rate * dt;
  c.wear[i] = pymin(100.0, c.wear[i]);
}
__device__ inline void weight_transfer(double lon, double lat, double speed, double out[4]) {
  double sw = CAR_MASS * GRAVITY_MS2, sfl = sw * 0.5, srl = sw * 0.5;
  double aero = 0.0;
  if (speed > 50.0) {
    double sf = P2(speed / 50.0);
    double calc = 0.12 * sf * CAR_MASS * GRAVITY_MS2;
    double mx = 1.5 * CAR_MASS * GRAVITY_MS2;
    aero = pymin(calc, mx);
  }
  double ar = aero * 0.6, af = aero * (1.0 - 0.6);
  double bf = sfl + af, br = srl + ar, te = sw + aero;
  double rl = lon * te * 0.02;
  double mf = bf * 0.95, mb = br * 0.95;
  double lt = rl > 0 ? pymin(rl, mf) : pymax(rl, -mb);
  double ft = bf - lt, rt = br + lt;
  double rlat = lat * te * 0.01;
  double mltf = (ft / 2.0) - 200.0, mltr = (rt / 2.0) - 200.0;
  double mlt = pymin(mltf, mltr);
  double latt = mlt > 0 ? pymax(-mlt, pymin(mlt, rlat)) : 0.0;
  double raw[4] = {ft / 2.0 - latt / 2.0, ft / 2.0 + latt / 2.0, rt / 2.0 - latt / 2.0, rt / 2.0 + latt / 2.0};
  double con[4], deficit = 0.0, excess = 0.0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (raw[i] < 50.0) { con[i] = 50.0; deficit += 50.0 - raw[i]; }
    else { con[i] = raw[i]; excess += raw[i] - 50.0; }
  }
  if (deficit > 0.0 && excess > 0.0) {
    double fct = deficit / excess;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (raw[i] >= 50.0) { double e = con[i] - 50.0; out[i] = pymax(50.0, con[i] - e * fct); }
      else out[i] = con[i];
    }
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) out[i] = con[i];
  }
}
__device__ inline void lateral_heating(const Car& c, double ff[4], double speed) {
  if (speed < 2.0) return;
  double shm = 1.0;
  if (c.slip > 5.0) { double ex = c.slip - 5.0; shm = 2.2 + (0.04 * P2(ex)); shm = pymin(shm, 8.0); }
  double base = c.lfm * 0.05 * shm;
  double flh = base * 0.5 / 2.0, rlh = base * 0.5 / 2.0;
  if (fabs(c.steer) > 0.01 && speed > 3.0) {
    int of, orr, inf, inr;
    if (c.steer < 0) { of = 0; orr = 2; inf = 1; inr = 3; }
    else { of = 1; orr = 3; inf = 0; inr = 2; }
    double ofb = c.load[of] * 0.001, orb = c.load[orr] * 0.001;
    ff[of] += flh * 1.5 + ofb;
    ff[orr] += rlh * 1.5 + orb;
    ff[inf] += flh * 0.5;
    ff[inr] += rlh * 0.5;
  } else { ff[0] += flh; ff[1] += flh; ff[2] += rlh; ff[3] += rlh; }
}
__device__ inline void update_friction(Car& c, double df) {
  double speed = (double)vlen(c.v);
  double rear, front;
  if (c.thr > 0.01 && speed > 50.0) { double fa = pymin(0.3, speed / 200.0); rear = df * (1.0 - fa); front = df * fa / 2.0; }
  else { rear = c.thr > 0.01 ? df : 0.0; front = 0.0; }
  double bf = 0.0;
  if (c.brk > 0.01) {
    double mbf = CAR_MASS * 14.0 * c.brk, base = mbf / 4.0;
    if (speed <= 1.0) { double sf = 0.05 + (1.0 - 0.05) * (speed / 1.0); bf = base * sf; }
    else bf = base;
  }
  double rf = 0.0;
  if (speed > 0.1) rf = ROLLING_RESISTANCE_FORCE / 4.0;
  double ff[4] = {front + bf + rf, front + bf + rf, rear / 2.0 + bf + rf, rear / 2.0 + bf + rf};
  lateral_heating(c, ff, speed);
#pragma unroll
  for (int i = 0; i < 4; ++i) c.fric[i] = ff[i];
}
__device__ __forceinline__ V2 OV(double x, double y) { return V((float)x, (float)y); }

// Car.update_physics (src/car.py:329-387) and helpers (:389-892)
__device__ inline void car_update_physics(const Params& P, Car& c, int n, const TrackDev& T) {
  const double dt = P.dt_d;
  c.thr = c.thr_in; c.brk = c.brk_in; c.steer = c.str_in * (45.0 * RAD_PER_DEG);
  {
    double target = 1000.0 + (800.0 * c.thr_in);
    double diff = target - c.rpm;
    c.rpm += diff * pymin(1.0, dt * 3000.0 / fabs(diff + 0.1));
    c.rpm = pymax(600.0, pymin(9500.0, c.rpm));
  }
  V2 fwd = V(c.xf.q.c * 1.0f - c.xf.q.s * 0.0f, c.xf.q.s * 1.0f + c.xf.q.c * 0.0f);
  {  // _apply_engine_force (:389-449)
    double speed = (double)vlen(c.v);
    double rpm = c.rpm < 1000.0 ? 1000.0 : (c.rpm > 9000.0 ? 9000.0 : c.rpm);
    double tf = rpm <= 5500.0 ? 0.7 + 0.3 * (rpm - 1000.0) / (5500.0 - 1000.0) : 1.0 - 0.6 * (rpm - 5500.0) / (9000.0 - 5500.0);
    double torque = CAR_MAX_TORQUE * tf * c.thr;
    double wheel = torque * 7.5;
    double tlf = wheel / 0.35;
    double ef;
    if (speed > 12.0) {
      double plf = (CAR_MAX_POWER * c.thr) / speed;
      if (speed <= 25.0) {
        double nsd = (speed - 12.0) / (25.0 - 12.0);
        double ex = 1.0 - exp(-2.0 * nsd);
        double blend = pymax(0.05, pymin(0.75, ex));
        ef = tlf * (1.0 - blend) + plf * blend;
      } else ef = tlf * (1.0 - 0.75) + plf * 0.75;
    } else ef = tlf;
    double grip = total_grip(c);
    double sfac = 1.0 - pymin(0.4, fabs(c.steer) * 1.5);
    double mx = CAR_MASS * GRAVITY_MS2 * grip * sfac;
    ef = pymin(ef, mx);
    double Fx = ef * (double)fwd.x, Fy = ef * (double)fwd.y;
    double rff = pymin(2000.0, fabs(ef) / 2.0);
    update_friction(c, rff);
    DBG(n, 0, ef); DBG(n, 1, Fx); DBG(n, 2, Fy); DBG(n, 3, speed); DBG(n, 4, c.rpm); DBG(n, 5, total_grip(c));

    float lx = (float)(-CAR_WHEELBASE / 2), ly = 0.0f;
    V2 pt = V((c.xf.q.c * lx - c.xf.q.s * ly) + c.xf.p.x, (c.xf.q.s * lx + c.xf.q.c * ly) + c.xf.p.y);
    apply_force(c, OV(Fx, Fy), pt);
  }
  PROFU(11);
  if (c.brk > 0.01) {  // _apply_brake_force (:451-469)
    double sfac = 1.0 - pymin(0.3, fabs(c.steer) * 1.5);
    double mbf = CAR_MASS * 14.0 * sfac;
    double bf = mbf * c.brk;
    double speed = (double)vlen(c.v);
    if (speed > 0.1) {
      double dx = -(double)c.v.x / speed, dy = -(double)c.v.y / speed;
      apply_force_center(c, OV(bf * dx, bf * dy));
      update_friction(c, 0.0);
    }
  }
  {  // drag (:471-484)
    double speed = (double)vlen(c.v);
    if (speed > 0.1) {
      double mag = DRAG_CONSTANT * speed * speed;
      double dx = -(double)c.v.x / speed, dy = -(double)c.v.y / speed;
      apply_force_center(c, OV(mag * dx, mag * dy));
    }
  }
  {  // rolling (:486-500)
    double speed = (double)vlen(c.v);
    if (speed > 0.1) {
      double rr = ROLLING_RESISTANCE_FORCE;
      double dx = -(double)c.v.x / speed, dy = -(double)c.v.y / speed;
      apply_force_center(c, OV(rr * dx, rr * dy));
    }
  }
  double alon, alat;
  {  // _get_acceleration (:832-892); history ring in HBM, summed oldest -> newest like Python's sum()
    double cvx = c.v.x, cvy = c.v.y;
    double ax = (cvx - c.pvx) / dt, ay = (cvy - c.pvy) / dt;
    float rtx = c.xf.q.c * 0.0f - c.xf.q.s * 1.0f, rty = c.xf.q.s * 0.0f + c.xf.q.c * 1.0f;
    double lon = ax * fwd.x + ay * fwd.y, lat = ax * rtx + ay * rty;
    lon = pymax(-12.0, pymin(12.0, lon));
    lat = pymax(-12.0, pymin(12.0, lat));
    // history as a ring in HBM (acc_head = slot of the oldest sample): the 10 slots are loaded oldest-first
    // (independent loads, issued together), the new sample is appended in registers and summed oldest ->
    // newest like Python's sum(), and only its slot is written back (16 B per car-step, not the whole deque)
    double* acc = P.acc;
    const size_t N = P.N;
    const int h0 = c.acc_head;
    double hl[10], ht[10];
#pragma unroll
    for (int q = 0; q < 10; ++q) {
      const int sq = h0 + q < 10 ? h0 + q : h0 + q - 10;
      hl[q] = acc[(size_t)(2 * sq) * N + n]; ht[q] = acc[(size_t)(2 * sq + 1) * N + n];
    }
    int wslot;
    if (c.acc_len == 10) {   // deque(maxlen=10).append: the oldest sample drops out
#pragma unroll
      for (int q = 0; q < 9; ++q) { hl[q] = hl[q + 1]; ht[q] = ht[q + 1]; }
      hl[9] = lon; ht[9] = lat;
      wslot = h0;
      c.acc_head = h0 + 1 < 10 ? h0 + 1 : 0;
    } else {
#pragma unroll
      for (int q = 0; q < 10; ++q) if (q == c.acc_len) { hl[q] = lon; ht[q] = lat; }
      wslot = h0 + c.acc_len < 10 ? h0 + c.acc_len : h0 + c.acc_len - 10;
      c.acc_len++;
    }
    double s0 = 0.0, s1 = 0.0;
#pragma unroll
    for (int q = 0; q < 10; ++q) if (q < c.acc_len) { s0 += hl[q]; s1 += ht[q]; }
    acc[(size_t)(2 * wslot) * N + n] = lon; acc[(size_t)(2 * wslot + 1) * N + n] = lat;
    alon = s0 / c.acc_len; alat = s1 / c.acc_len;
    DBG(n, 6, alon); DBG(n, 7, alat);

    c.pvx = cvx; c.pvy = cvy;
  }
  PROFU(12);
  {  // TyreManager.update (src/tyre_manager.py:78-97)
    double speed = (double)vlen(c.v);
    double loads[4];
    weight_transfer(alon, alat, speed, loads);
    double fr[4] = {c.fric[0], c.fric[1], c.fric[2], c.fric[3]};
    DBG(n, 8, fr[0]); DBG(n, 9, fr[2]);

#pragma unroll
    for (int i = 0; i < 4; ++i) c.load[i] = loads[i];
#pragma unroll
    for (int i = 0; i < 4; ++i) tyre_update(c, i, dt, loads[i], fr[i], speed, alat, c.slip);
  }
  PROFU(13);
  {  // _apply_lateral_tire_forces (:635-700)
    double speed = (double)vlen(c.v);
    if (speed > 0.05) {
      c.lfm = 0.0; c.slip = 0.0;
      double cs = (double)vlen(c.v);
      if (!(cs < 0.05)) {
        double fx = fwd.x, fy = fwd.y;
        double vnx = (double)c.v.x / cs, vny = (double)c.v.y / cs;
        double cr = vnx * fy - vny * fx, dt_ = vnx * fx + vny * fy;
        double sr = atan2(fabs(cr), dt_);
        c.slip = fabs(sr) * DEG_PER_RAD;
        double dvx = fx * cs, dvy = fy * cs;
        double ex = dvx - (double)c.v.x, ey = dvy - (double)c.v.y;
        double aff = CAR_MASS * 5.0;
        double cx = ex * aff, cy = ey * aff;
        double grip = total_grip(c);
        double pbf = CAR_MASS * GRAVITY_MS2 * grip * 1.0;
        double mf = pymin(30000.0 * grip, pbf);
        double fm = PH(P2(cx) + P2(cy));
        DBG(n, 10, cs); DBG(n, 11, cx); DBG(n, 12, cy); DBG(n, 13, fm); DBG(n, 14, c.slip);

        if (fm > mf) { double sc = mf / fm; cx = cx * sc; cy = cy * sc; fm = mf; }
        c.lfm = fm;
        apply_force_center(c, OV(cx, cy));
      }
    }
  }
  DBG(n, 15, c.force.x); DBG(n, 16, c.force.y); DBG(n, 17, c.torque);
  apply_torque(c, (float)(-(double)c.w * CAR_MASS * 4.0));   // _apply_angular_damping (:502-507)
  if (!(fabs(c.bank) < 0.1)) {  // _apply_banking_forces (:509-566)
    double speed = (double)vlen(c.v);
    if (!(speed < 1.0)) {
      // lateral assist per segment precomputed on the host with the reference's math.sin
      double la = 0.0; bool found = false;
      for (int k = 0; k < T.nseg; ++k) if (T.segs[k].banking == c.bank) { la = T.segs[k].la; found = true; break; }
      if (!found) { double br = c.bank * RAD_PER_DEG; la = (CAR_MASS * 9.81) * sin(fabs(br)) * 0.3; }
      if (!(fabs(la) < 1.0) && speed > 5.0) {
        double vx = (double)c.v.x / speed, vy = (double)c.v.y / speed;
        double fdx = -vy, fdy = vx;
        double sg = copysign(1.0, c.bank);
        apply_force_center(c, OV(fdx * la * sg, fdy * la * sg));
      }
    }
  }
  if (fabs(c.steer) > 0.01) {  // _apply_steering_torque (:568-584)
    double speed = (double)vlen(c.v);
    if (speed > 0.1) {
      double dav = speed * tan(c.steer) / CAR_WHEELBASE;
      double err = dav - (double)c.w;
      apply_torque(c, (float)(err * CAR_MASS * 0.8));
    }
  }
}

// ------------------------------------------------------------------ track lookups
__device__ inline double banking_at(const TrackDev& T, double px, double py) {
  double best = INFINITY; int bi = -1;
  for (int k = 0; k < T.nseg; ++k) {
    const DSeg& s = T.segs[k];
    double ll = P2(s.ex - s.sx) + P2(s.ey - s.sy), d;
    if (ll == 0) d = sqrt(P2(px - s.sx) + P2(py - s.sy));
    else {
      double tt = ((px - s.sx) * (s.ex - s.sx) + (py - s.sy) * (s.ey - s.sy)) / ll;
      tt = pymax(0.0, pymin(1.0, tt));
      double qx = s.sx + tt * (s.ex - s.sx), qy = s.sy + tt * (s.ey - s.sy);
      d = sqrt(P2(px - qx) + P2(py - qy));
    }
    if (d < best) { best = d; bi = k; }
  }
  return bi >= 0 ? T.segs[bi].banking : 0.0;
}
__device__ inline double track_progress(const TrackDev& T, double px, double py) {
  double best = INFINITY; int bi = 0; double bx = 0, by = 0;
  for (int k = 0; k < T.nseg; ++k) {
    const DSeg& s = T.segs[k];
    double dx = s.ex - s.sx, dy = s.ey - s.sy, ll = dx * dx + dy * dy, qx, qy;
    if (ll < 1e-6) { qx = s.sx; qy = s.sy; }
    else {
      double tt = pymax(0.0, pymin(1.0, ((px - s.sx) * dx + (py - s.sy) * dy) / ll));
      qx = s.sx + tt * dx; qy = s.sy + tt * dy;
    }
    double d2 = P2(px - qx) + P2(py - qy);
    if (d2 < best) { best = d2; bi = k; bx = qx; by = qy; }
  }
  const DSeg& s = T.segs[bi];
  return T.prefix[bi] + sqrt(P2(bx - s.sx) + P2(by - s.sy));
}
__device__ inline bool on_startline(const TrackDev& T, double px, double py) {
  const DSeg& s = T.segs[T.startline];
  double dx = s.ex - s.sx, dy = s.ey - s.sy, ll = dx * dx + dy * dy, d;
  if (ll < 1e-6) d = sqrt(P2(px - s.sx) + P2(py - s.sy));
  else {
    double tt = pymax(0.0, pymin(1.0, ((px - s.sx) * dx + (py - s.sy) * dy) / ll));
    double qx = s.sx + tt * dx, qy = s.sy + tt * dy;
    d = sqrt(P2(px - qx) + P2(py - qy));
  }
  return d <= (s.width / 2.0);
}

// f32 screen of the chord searches above, for the logic kernel (segments staged in LDS as
// (sx, sy, ex - sx, ey - sy) plus 1 / |e - s|^2, 0 for chords shorter than 1e-3 m).  A screened
// distance is within screen_eps of the f64 one (f32 rounding of coordinates and of the projection:
// ~1e-3 m on km-sized tracks; the term in |p| covers far-off cars), so a chord whose screened
// distance exceeds the screened minimum by more than 2 screen_eps is strictly farther than the
// screened minimiser in f64 too: it can neither be nor tie the reference's nearest chord.  The
// exact f64 evaluation (with the reference's strict '<', in index order) runs on the rest only.
struct ChordScreen { const float4* g; const float* rll; int n; };
__device__ __forceinline__ float screen_eps(float x, float y) { return 0.05f + 4e-6f * (fabsf(x) + fabsf(y)); }
__device__ __forceinline__ float screen_d2(const ChordScreen& S, int k, float x, float y) {
  const float4 g = S.g[k];
  const float rx = x - g.x, ry = y - g.y;
  const float tt = fminf(1.0f, fmaxf(0.0f, (rx * g.z + ry * g.w) * S.rll[k]));
  const float ex = rx - tt * g.z, ey = ry - tt * g.w;
  return ex * ex + ey * ey;
}
// The chords that pass the screen, as a bit mask (bit k: chord k; MAX_SEG <= 64): a chord whose squared screened
// distance exceeds cut = (sqrt(min) + 2 screen_eps)^2 (x 1.0001) cannot be the nearest one.  The first SCREEN_R chords'
// loads are issued together and their distances kept in registers for the mask (the bundled tracks have 7-9 chords;
// a loop over the rest).
#define SCREEN_R 16
static_assert(MAX_SEG <= 64, "screen_candidates keeps one bit per chord");
__device__ inline uint64_t screen_candidates(const ChordScreen& S, float x, float y) {
  float d[SCREEN_R], m = INFINITY;
#pragma unroll
  for (int k = 0; k < SCREEN_R; ++k) { d[k] = k < S.n ? screen_d2(S, k, x, y) : INFINITY; m = fminf(m, d[k]); }
  for (int k = SCREEN_R; k < S.n; ++k) m = fminf(m, screen_d2(S, k, x, y));
  const float r = __builtin_amdgcn_sqrtf(m) + 2.0f * screen_eps(x, y);
  const float cut = r * r * 1.0001f;
  uint64_t mask = 0;
#pragma unroll
  for (int k = 0; k < SCREEN_R; ++k) if (k < S.n && !(d[k] > cut)) mask |= 1ull << k;
  for (int k = SCREEN_R; k < S.n; ++k) if (!(screen_d2(S, k, x, y) > cut)) mask |= 1ull << k;
  return mask;
}
// track_progress restricted to the screen's candidate chords (same results: the exact search in index order)
__device__ inline double track_progress_screened(const TrackDev& T, uint64_t cand, double px, double py) {
  double best = INFINITY; int bi = 0; double bx = 0, by = 0;
  for (uint64_t mk = cand; mk; mk &= mk - 1) {
    const int k = __builtin_ctzll(mk);
    const DSeg& s = T.segs[k];
    double dx = s.ex - s.sx, dy = s.ey - s.sy, ll = dx * dx + dy * dy, qx, qy;
    if (ll < 1e-6) { qx = s.sx; qy = s.sy; }
    else {
      double tt = pymax(0.0, pymin(1.0, ((px - s.sx) * dx + (py - s.sy) * dy) / ll));
      qx = s.sx + tt * dx; qy = s.sy + tt * dy;
    }
    double d2 = P2(px - qx) + P2(py - qy);
    if (d2 < best) { best = d2; bi = k; bx = qx; by = qy; }
  }
  const DSeg& s = T.segs[bi];
  return T.prefix[bi] + sqrt(P2(bx - s.sx) + P2(by - s.sy));
}
// banking_at and track_progress over the candidate chords in one pass (each search's own arithmetic and strict '<' in
// index order, so the same results; the two chains interleave)
__device__ inline double bank_and_progress_screened(const TrackDev& T, uint64_t cand, double px, double py, double& prog) {
  double bbest = INFINITY; int bbi = -1;
  double pbest = INFINITY; int pbi = 0; double bx = 0, by = 0;
  for (uint64_t mk = cand; mk; mk &= mk - 1) {
    const int k = __builtin_ctzll(mk);
    const DSeg& s = T.segs[k];
    {   // banking_at
      double ll = P2(s.ex - s.sx) + P2(s.ey - s.sy), d;
      if (ll == 0) d = sqrt(P2(px - s.sx) + P2(py - s.sy));
      else {
        double tt = ((px - s.sx) * (s.ex - s.sx) + (py - s.sy) * (s.ey - s.sy)) / ll;
        tt = pymax(0.0, pymin(1.0, tt));
        double qx = s.sx + tt * (s.ex - s.sx), qy = s.sy + tt * (s.ey - s.sy);
        d = sqrt(P2(px - qx) + P2(py - qy));
      }
      if (d < bbest) { bbest = d; bbi = k; }
    }
    {   // track_progress
      double dx = s.ex - s.sx, dy = s.ey - s.sy, ll = dx * dx + dy * dy, qx, qy;
      if (ll < 1e-6) { qx = s.sx; qy = s.sy; }
      else {
        double tt = pymax(0.0, pymin(1.0, ((px - s.sx) * dx + (py - s.sy) * dy) / ll));
        qx = s.sx + tt * dx; qy = s.sy + tt * dy;
      }
      double d2 = P2(px - qx) + P2(py - qy);
      if (d2 < pbest) { pbest = d2; pbi = k; bx = qx; by = qy; }
    }
  }
  const DSeg& sp = T.segs[pbi];
  prog = T.prefix[pbi] + sqrt(P2(bx - sp.sx) + P2(by - sp.sy));
  return bbi >= 0 ? T.segs[bbi].banking : 0.0;
}
// on_startline, decided by the screen unless the screened distance is within screen_eps of width / 2
__device__ inline bool on_startline_screened(const TrackDev& T, const ChordScreen& S, double px, double py) {
  const float x = (float)px, y = (float)py;
  const float d = __builtin_amdgcn_sqrtf(screen_d2(S, T.startline, x, y));
  const float h = (float)(T.segs[T.startline].width / 2.0), e = screen_eps(x, y);
  if (d < h - e) return true;
  if (d > h + e) return false;
  return on_startline(T, px, py);
}
// LapTimer.update (src/lap_timer.py:95-272)
// lt_has_pos: bit 0 = a previous position is recorded, bit 1 = that position was on the start line
// (LapTimer._is_on_start_line(previous_position), src/lap_timer.py:193, evaluated when it was current)
__device__ inline bool lap_update(const TrackDev& T, const ChordScreen& S, Car& c, double px, double py, double sim) {
  if (c.lt_timing) c.lt_cur = sim - c.lt_start;
  if (c.lt_has_pos) {
    double dx = px - c.lt_px, dy = py - c.lt_py, d = sqrt(dx * dx + dy * dy);
    if (d < 50.0) c.lt_dist += d;
  }
  bool done = false;
  const bool now = T.startline >= 0 && on_startline_screened(T, S, px, py);
  if (T.startline >= 0 && c.lt_has_pos) {
    const bool before = (c.lt_has_pos & 2) != 0;
    if (now && !before) {
      if (c.lt_crossed && c.lt_timing) {
        double minlap = T.total_length > 0 ? T.total_length * 0.95 : 100.0;
        if (c.lt_cur < 10.0) {
        } else if (c.lt_dist < minlap) {
        } else {
          double ct = c.lt_cur;
          c.lt_last = ct; c.lt_has_last = 1;
          if (!c.lt_has_best || ct < c.lt_best) { c.lt_best = ct; c.lt_has_best = 1; }
          c.lt_start = sim; c.lt_cur = 0.0; c.lt_timing = 1;
          c.lt_laps += 1; c.lt_dist = 0.0;
          done = true;
        }
      } else if (!c.lt_crossed) {
        c.lt_crossed = 1; c.lt_timing = 1; c.lt_start = sim; c.lt_cur = 0.0; c.lt_dist = 0.0;
      }
    }
  }
  c.lt_px = px; c.lt_py = py; c.lt_has_pos = now ? 3 : 1;
  return done;
}

// ------------------------------------------------------------------ distance sensors (src/distance_sensor.py:71-117)
// 16 rays x the walls in LDS.  The reference result per ray is the minimum over walls
// of the exact b2PolygonShape::RayCast fraction (maxFraction 1, p2 fixed), so any cull
// that provably keeps every wall that can hit a ray gives the identical minimum.
// Cull, per wall: (1) range -- the wall's bounding circle (radius R incl. margin) must
// reach within 250 m; (2) angle -- from the car the circle subtends
// [phi - asin(R/d), phi + asin(R/d)]; only rays whose direction falls inside (plus a
// 2e-3 rad guard for the approximate atan2 / f32 ray directions) are tested exactly.
// A wall at distance d cannot beat the current best of a ray if d - R exceeds it.
// Per-ray state (best fraction, f32 endpoint) lives in LDS so the ray loop can index
// it dynamically: rs = [3][16][BLOCK] floats of this workgroup.
__device__ __forceinline__ float atan2_approx(float y, float x) {   // |err| < 1.2e-5 rad
  float ax = fabsf(x), ay = fabsf(y);
  float mx = fmaxf(ax, ay), mn = fminf(ax, ay);
  float t = mx > 0.0f ? mn * __builtin_amdgcn_rcpf(mx) : 0.0f;
  float s2 = t * t;
  float r = ((((0.0208351f * s2 - 0.0851330f) * s2 + 0.1801410f) * s2 - 0.3302995f) * s2 + 0.9998660f) * t;
  if (ay > ax) r = 1.57079637f - r;
  if (x < 0.0f) r = 3.14159274f - r;
  return y < 0.0f ? -r : r;
}

// CarPhysics._check_wall_collision AABB query (src/car_physics.py:470-524)
__device__ inline bool query_on_wall(const WallSet& S, double px, double py, double radius) {
  const LWall* W = S.W;
  Aabb q; q.lo = V((float)(px - radius), (float)(py - radius)); q.hi = V((float)(px + radius), (float)(py + radius));
  V2 center = V((float)px, (float)py);
  int beg = 0, end = S.nw;
  const uint16_t* list = nullptr;
  if (radius <= (double)S.bp.reach - 0.1 && grid_list(S.bp, 0.5f * (q.lo.x + q.hi.x), 0.5f * (q.lo.y + q.hi.y), beg, end))
    list = S.bp.idx;
  else { beg = 0; end = S.nw; }
  for (int kk = beg; kk < end; ++kk) {
    const int jw = list ? (int)ldg(list + kk) : kk;
    if (!overlap(fat_box(ldg(S.fat + jw)), q)) continue;
    const LWall wl = ldg(W + jw);
    Xf xf = wall_xf(wl);
    Poly p; make_box(&p, wl.hx, wl.hy);
    V2 pl = rmulT(xf.q, vsub(center, xf.p));
    bool inside = true;
    for (int i = 0; i < 4; ++i) { if (vdot(pn(&p, i), vsub(pl, pv(&p, i))) > 0.0f) { inside = false; break; } }
    if (inside) return true;
    for (int i = 0; i < 4; ++i) {
      V2 v = xmul(xf, pv(&p, i));
      double dx = px - (double)v.x, dy = py - (double)v.y;
      if (PH(dx * dx + dy * dy) < radius) return true;
    }
  }
  return false;
}

// CarEnv._get_multi_obs for one car (src/car_env.py:891-956): obs[0:22] (the 16 sensor
// values obs[22:38] are written by sensor_kernel from the pose handed over in P.pose)
__device__ inline void car_obs(const Car& c, float* o) {
  double px = c.xf.p.x, py = c.xf.p.y, vx = c.v.x, vy = c.v.y, ang = c.a, av = c.w;
  o[0] = (float)npclip(px / 10000.0, -1, 1); o[1] = (float)npclip(py / 10000.0, -1, 1);
  o[2] = (float)npclip(vx / 111.1, -1, 1); o[3] = (float)npclip(vy / 111.1, -1, 1);
  o[4] = (float)npclip(PH(P2(vx) + P2(vy)) / 111.1, 0, 1);
  o[5] = (float)npclip(ang / PI_D, -1, 1); o[6] = (float)npclip(av / 10.0, -1, 1);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    o[7 + i] = (float)npclip(c.load[i] / MAX_TYRE_LOAD, 0, 1);
    o[11 + i] = (float)npclip(c.temp[i] / 200.0, 0, 1);
    o[15 + i] = (float)npclip(c.wear[i] / 100.0, 0, 1);
  }
  double ci = c.imp_present ? c.imp : 0.0, imp = 0.0, ca = 0.0;
  if (!(ci < 100.0)) {   // CarPhysics.get_collision_data (src/car_physics.py:386-425)
    imp = ci;
    if (c.nact > 0) {
      double na = atan2((double)c.act_n[1], (double)c.act_n[0]);
      double a = na - (double)c.a;
      while (a > PI_D) a -= 2 * PI_D;
      while (a < -PI_D) a += 2 * PI_D;
      ca = a;
    }
  }
  o[19] = (float)npclip(imp / 50000.0, 0, 1); o[20] = (float)npclip(ca / PI_D, -1, 1);
  o[21] = (float)npclip(c.cum_impact / 250000.0, 0, 1);
}
// sensor hand-off modes (bits): A -> obs, A -> terminal_obs, B -> obs
#define PM_A_OBS 1
#define PM_A_TERM 2
#define PM_B_OBS 4
__device__ __forceinline__ float4 car_pose(const Car& c, int mode) {
  return make_float4(c.xf.p.x, c.xf.p.y, c.a, __int_as_float(mode));
}
// pose hand-off slot k (n: pass A, N + n: pass B) with the f64 cos / sin of the angle the rays rotate
__device__ __forceinline__ void set_pose(const Params& P, size_t k, const Car& c, int mode) {
  P.pose[k] = car_pose(c, mode);
  double s0, c0;
  sincos((double)c.a, &s0, &c0);
  P.pose_cs[k] = make_double2(c0, s0);
}

// ------------------------------------------------------------------ reset (src/car_env.py:316-535)
__device__ inline void car_reset(const Params& P, Car& c, int n, bool fresh, const WallSet& S, const TrackDev& T) {
  V2 p = OV(P.start_x, P.start_y); float a = P.start_angle;
  if (P.car_contact) {   // extension only: a staggered grid (rows of 2, 8 m apart, +-3 m), so cars do not start overlapped
    const int i = n % P.C;
    const Rot q = rot_set(a);
    p = vadd(p, rmul(q, V(-8.0f * (float)(i >> 1), (i & 1) ? -3.0f : 3.0f)));
    if (P.C == 1) p = OV(P.start_x, P.start_y);
  }
  if (fresh) {   // Car() + CarPhysics(car, track): new b2World (src/car_physics.py:74-107)
    c.xf.q = rot_set(a); c.xf.p = p;
    c.c = xmul(c.xf, zero2()); c.a = a; c.c0 = c.c; c.a0 = a;
    c.v = zero2(); c.w = 0.0f; c.sleep = 0.0f; c.awake = 1; c.invdt0 = 0.0f;
    c.force = zero2(); c.torque = 0.0f; c.alpha0 = 0.0f;
    Poly cp; make_box(&cp, CAR_HX, CAR_HY);
    Aabb ab = poly_aabb(&cp, c.xf);
    V2 r = V(AABB_EXT, AABB_EXT);
    c.fat.lo = vsub(ab.lo, r); c.fat.hi = vadd(ab.hi, r);
    c.nct = 0; c.overflow = 0; c.moved = 1;
    find_new_contacts(c, S);
    c.bank = 0.0;
  } else {       // CarPhysics.reset_car + Car.reset (src/car_physics.py:550-571, src/car.py:1027-1058)
    set_transform(c, S, p, c.a);
    set_transform(c, S, c.xf.p, a);
    set_transform(c, S, p, c.a);
    set_transform(c, S, c.xf.p, a);
    c.v = zero2(); c.w = 0.0f;
  }
  c.rpm = 1000.0;
#pragma unroll
  for (int i = 0; i < 4; ++i) { c.temp[i] = 80.0; c.wear[i] = 0.0; c.load[i] = (CAR_MASS * GRAVITY_MS2 * 0.5) / 2.0; }
  c.pvx = c.pvy = 0.0; c.acc_len = 0; c.acc_head = 0; c.lfm = 0.0; c.slip = 0.0;
  c.nact = 0; c.imp_present = 0; c.imp = 0.0;
  c.lt_timing = 0; c.lt_start = 0.0; c.lt_cur = 0.0; c.lt_has_last = c.lt_has_best = 0; c.lt_last = c.lt_best = 0.0;
  c.lt_crossed = 0; c.lt_has_pos = 0; c.lt_px = c.lt_py = 0.0; c.lt_laps = 0; c.lt_dist = 0.0;
  c.disabled = 0; c.just_disabled = 0; c.cum_impact = 0.0; c.stuck_dur = 0.0; c.has_stuck_start = 0;
  c.stuck_sx = c.stuck_sy = 0.0;
  c.prev_px = c.xf.p.x; c.prev_py = c.xf.p.y;
  c.back = c.prev_back = 0.0; c.first_step = 1; c.prev_laps = 0; c.cum_reward = 0.0f; c.cum_reward_info = 0.0f;
  c.prog_hist = track_progress(T, c.xf.p.x, c.xf.p.y);
  c.imp_at_obs = 0.0;
}

// ------------------------------------------------------------------ the fused step
extern __shared__ __attribute__((aligned(16))) unsigned char smem[];


// Sensor kernel: LPC lanes per car, BLOCK / LPC cars of one track per workgroup.
// The candidate list of the car's cell (WallGrid sn) holds wall GROUPS (runs of adjacent
// walls with a bounding circle), nearest first; lane r of a car takes groups r, r+LPC, ...
// Per group: range test, angular ray mask (as for single walls), then the rays whose
// current best (shared by the car's lanes in LDS, atomicMin) is already closer than the
// group are dropped; surviving rays are tested per wall with the bounding-circle cull and
// the exact b2PolygonShape::RayCast.  The result is the minimum over every wall that can
// hit each ray, i.e. the reference's value, whatever the visiting order.
#ifndef SENSOR_LPC
#define SENSOR_LPC 4
#endif
__device__ __forceinline__ float sensor_value(float best) {   // DistanceSensor distance -> obs (src/car_env.py:946)
  double hd = best <= 1.0f ? (double)best * 250.0 : 250.0;
  float d32 = (float)hd;
  float v = fdiv_cr(d32, 250.0f);
  return v < 0.0f ? 0.0f : (v > 1.0f ? 1.0f : v);
}

// ray offsets of DistanceSensor (nascar_rays.h)
// The table lives in a device buffer (Params::ray_cs, filled at nascar_create) and is read with one
// indexed load: as a __constant__ array hipcc materialised all 32 values in registers per lane,
// selected by the (lane-varying) ray index, and spilled them.
static const double h_ray_cs[16][2] = NASCAR_RAY_CS_INIT;
__device__ __forceinline__ V2 ray_end(const Params& P, double px, double py, double ang, double c0, double s0, int i,
                                      double& dx, double& dy) {
  float fx, fy;
  ray_end_f32(px, py, ang, c0, s0, i, (const double (*)[2])P.ray_cs, dx, dy, fx, fy);
  return V(fx, fy);
}
__device__ __forceinline__ V2 ray_end_k(double px, double py, double ang, double c0, double s0, int i, double2 rk,
                                        double& dx, double& dy) {   // rk = ray_cs[i], loaded by the caller
  float fx, fy;
  ray_end_f32_k(px, py, ang, c0, s0, i, rk.x, rk.y, dx, dy, fx, fy);
  return V(fx, fy);
}

// rays (pi/8 apart, ray i along ang - i*pi/8) that can meet a circle (center r from the car, radius R)
__device__ __forceinline__ unsigned ray_mask(float rx, float ry, float d, float R, float angf) {
  if (d <= R * 1.0001f + 0.01f) return 0xFFFFu;
  const float K = 2.54647909f;   // 8 / pi
  const float x = R * __builtin_amdgcn_rcpf(d) * 1.0001f;
  const float half = fminf(x * (1.0f + 0.5708f * x * x), 1.5708f) + 2e-3f;   // >= asin(R/d) + guard
  float u = (angf - atan2_approx(ry, rx)) * K;                                  // ray-index coordinate
  u = u - 16.0f * floorf(u * 0.0625f);
  const float w = half * K;
  const int lo = (int)ceilf(u - w), hi = (int)floorf(u + w);
  const int cnt = hi - lo + 1;
  if (cnt <= 0) return 0u;
  if (cnt >= 16) return 0xFFFFu;
  const unsigned m = (1u << cnt) - 1u;
  return ((m << (lo & 15)) | (m >> (16 - (lo & 15)))) & 0xFFFFu;
}

// Rays that can meet a long thin wall: the box lies inside the capsule of its centre line
// (end points A, B) with radius rr; seen from p1 the capsule spans the arc between the
// directions to A and B (< pi when p1 is off the segment) widened by asin(rr / dist).
// dseg returns the point-to-segment distance (occlusion bound).
__device__ __forceinline__ unsigned seg_ray_mask(float ax, float ay, float bx, float by, float rr, float angf, float& dseg) {
  const float sx = bx - ax, sy = by - ay;
  const float ll = sx * sx + sy * sy;
  float tt = ll > 0.0f ? -(ax * sx + ay * sy) * __builtin_amdgcn_rcpf(ll) : 0.0f;
  tt = fminf(1.0f, fmaxf(0.0f, tt));
  const float qx = ax + tt * sx, qy = ay + tt * sy;
  dseg = __builtin_amdgcn_sqrtf(qx * qx + qy * qy);
  if (dseg <= rr * 1.0001f + 0.05f) return 0xFFFFu;
  const float K = 2.54647909f;   // 8 / pi
  const float x = rr * __builtin_amdgcn_rcpf(dseg) * 1.0001f;
  const float half = fminf(x * (1.0f + 0.5708f * x * x), 1.5708f) + 2e-3f;   // >= asin(rr / dseg) + guard
  float ua = (angf - atan2_approx(ay, ax)) * K, ub = (angf - atan2_approx(by, bx)) * K;
  ua = ua - 16.0f * floorf(ua * 0.0625f);
  ub = ub - 16.0f * floorf(ub * 0.0625f);
  if (ub < ua) { const float tmp = ua; ua = ub; ub = tmp; }
  if (ub - ua > 8.0f) { const float tmp = ua + 16.0f; ua = ub; ub = tmp; }   // take the short arc
  const float w = half * K;
  const int lo = (int)ceilf(ua - w), hi = (int)floorf(ub + w);
  const int cnt = hi - lo + 1;
  if (cnt <= 0) return 0u;
  if (cnt >= 16) return 0xFFFFu;
  const unsigned m = (1u << cnt) - 1u;
  return ((m << (lo & 15)) | (m >> (16 - (lo & 15)))) & 0xFFFFu;
}

template <int LPC>
#ifndef SENSOR_WPE
#define SENSOR_WPE 6   // 80 VGPRs: all 5 464 waves of the 8192x10 bench resident at once (measured best of 4/5/6)
#endif
__global__ void __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(SENSOR_WPE))) sensor_kernel(Params P, float* obs,
                                                                                                        float* terminal_obs, int passes) {
  constexpr int CPW = BLOCK / LPC;          // cars per workgroup
  constexpr int RPL = 16 / LPC;             // rays whose end points / outputs a lane owns
  PROF_B0(P.blk0 * ((SBLOCK + CPW - 1) / CPW));   // profile builds: stamp rows of the whole grid (launch_sensors_impl's sub)
  PROFS_RT(14);
  PROFS(0);
  __shared__ float s_p2[CPW * 32];          // [car][ray][x, y]: f32 ray end points (exact test)
  __shared__ unsigned s_best[CPW * 16];     // [car][ray]: best fraction so far (float bits, >= 0)
  float4* swa = (float4*)smem;
  constexpr int SUB = (SBLOCK + CPW - 1) / CPW;   // sensor workgroups per step-kernel workgroup
  const int bx = blockIdx.x, b = bx / SUB + P.blk0, sub = bx % SUB;
  const int t = threadIdx.x, lc = t / LPC, r = t - lc * LPC;
  const int C = P.C;
  const int slot = sub * CPW + lc;          // car slot within the step kernel's workgroup b
  const int el = slot / C, car = slot - el * C;
  const int env = blk_env_of(P, el, b * P.epb + el);
  if (blk_empty(P, b)) return;   // an empty workgroup of a device-built block map (random-track mode)
  const TrackDev T = P.tracks[blk_track_of(P, b)];
  const int nw = T.nwall, ng = T.ngroup;
  // walls and groups read straight from the track's global image (L1/L2-resident, shared by every
  // workgroup): no staging, no dynamic LDS
  (void)swa; (void)nw;
  const float4* __restrict__ swall = T.swall;
#define SW_A(j) swall[2 * (j)]
#define SW_B(j) swall[2 * (j) + 1]
  for (int g = t; g < ng; g += BLOCK) swa[g] = T.groups[g];   // groups (2-4 KB) staged in LDS; the barrier below publishes them
#define SW_G(g) swa[g]
  const int n = env >= 0 ? env * C + car : 0;
  float4 pa = make_float4(0.f, 0.f, 0.f, 0.f), pb = pa;
  int mode = 0;   // A bits from pose[n], the B bit from pose[N + n]
  if (env >= 0) {
    if (passes & 1) { pa = P.pose[n]; mode = __float_as_int(pa.w) & (PM_A_OBS | PM_A_TERM); }
    if ((passes & 2) && P.reset_env[env]) { pb = P.pose[P.N + n]; mode |= __float_as_int(pb.w) & PM_B_OBS; }
  }
  PROFS(1);
  unsigned* best = s_best + lc * 16;
  const float* p2s = s_p2 + lc * 32;
  for (int pass = (passes & 1) ? 0 : 1; pass < ((passes & 2) ? 2 : 1); ++pass) {
    const bool active = env >= 0 && (pass == 0 ? (mode & (PM_A_OBS | PM_A_TERM)) != 0 : (mode & PM_B_OBS) != 0);
    const float4 ps = pass == 0 ? pa : pb;
    const V2 p1 = V(ps.x, ps.y);
    const double px = ps.x, py = ps.y, ang = ps.z;
    double s0 = 0.0, c0 = 1.0;
    if (active) { const double2 cs = P.pose_cs[pass == 0 ? (size_t)n : (size_t)P.N + n]; c0 = cs.x; s0 = cs.y; }
#pragma unroll
    for (int q = 0; q < RPL; ++q) {
      const int i = r * RPL + q;
      if (active) {
        double dx, dy;
        const V2 p2 = ray_end(P, px, py, ang, c0, s0, i, dx, dy);
        s_p2[(lc * 16 + i) * 2] = p2.x; s_p2[(lc * 16 + i) * 2 + 1] = p2.y;
        (void)dx; (void)dy;
      }
      s_best[lc * 16 + i] = __float_as_uint(2.0f);
    }
    if (pass == 0) PROFS(2);
    __syncthreads();   // also publishes the staged walls / groups on pass 0
    if (pass == 0) PROFS(3);
    if (active) {
      int beg = 0, end = ng;
      const uint16_t* list = nullptr;
      if (grid_list(T.sn, p1.x, p1.y, beg, end)) list = T.sn.idx;
      else { beg = 0; end = ng; }
      const float angf = ps.z;
#ifdef NASCAR_PROFILE
      int c_vis = 0, c_rng = 0, c_open = 0, c_wr = 0, c_ex = 0, c_walls = 0;
#define CNT(x) (x)++
#else
#define CNT(x) do { } while (0)
#endif
      for (int kk = beg + r; kk < end; kk += LPC) {
        CNT(c_vis);
        const float4 G = SW_G(list ? (int)list[kk] : kk);
        const float grx = G.x - p1.x, gry = G.y - p1.y;
        const float d2 = grx * grx + gry * gry;
        if (d2 > (250.0f + G.z) * (250.0f + G.z)) continue;
        const float d = __builtin_amdgcn_sqrtf(d2);
        CNT(c_rng);
        unsigned mask;
        float dlo;   // lower bound of any hit fraction in the group
        if (G.z > 24.0f) {   // a single long (straight) wall: mask from its end points
          const int j = __float_as_int(G.w) & 0xFFFF;
          const float4 wa = SW_A(j), wb = SW_B(j);
          const float ex = wa.w * wb.y, ey = wa.w * wb.x;   // hx * (qc, qs)
          const float cx = wa.x - p1.x, cy = wa.y - p1.y;
          float dseg;
          mask = seg_ray_mask(cx - ex, cy - ey, cx + ex, cy + ey, wb.z * 1.4143f + 0.3f, angf, dseg);
          dlo = (dseg - (wb.z * 1.4143f + 0.3f)) * (1.0f / 250.0f) - 1e-4f;
        } else {
          mask = ray_mask(grx, gry, d, G.z, angf);
          dlo = (d - G.z) * (1.0f / 250.0f) - 1e-4f;
        }
        unsigned open = 0u;
        while (mask) {
          const int i = __builtin_ctz(mask);
          mask &= mask - 1u;
          if (!(dlo > __uint_as_float(best[i]))) open |= 1u << i;
        }
        if (!open) continue;
        CNT(c_open);
        const int first = __float_as_int(G.w) & 0xFFFF, cnt = __float_as_int(G.w) >> 16;
        for (int j = first; j < first + cnt; ++j) {
          const float4 wa = SW_A(j);
          const float4 wb = SW_B(j);
          const float rx = wa.x - p1.x, ry = wa.y - p1.y;
          const float R = wa.z;
          Rot q; q.s = wb.x; q.c = wb.y;
          const V2 l1 = rmulT(q, V(p1.x - wa.x, p1.y - wa.y));
          const float hx = wa.w, hy = wb.z;
          // numerators of the 4 faces depend only on p1 (b2Dot(normal_i, vertex_i - p1))
          const float n0 = 0.0f * ((-hx) - l1.x) + (-1.0f) * ((-hy) - l1.y);
          const float n1 = 1.0f * (hx - l1.x) + 0.0f * ((-hy) - l1.y);
          const float n2 = 0.0f * (hx - l1.x) + 1.0f * (hy - l1.y);
          const float n3 = (-1.0f) * ((-hx) - l1.x) + 0.0f * (hy - l1.y);
          unsigned m = open;
          CNT(c_walls);
          while (m) {
            const int i = __builtin_ctz(m);
            m &= m - 1u;
            const float bi = __uint_as_float(best[i]);
            CNT(c_wr);
            // direction from the f32 end point (cull only: error ~1e-7 rad, far inside the guards);
            // the end point is re-read by the exact cast below
            const float px2 = p2s[2 * i], py2 = p2s[2 * i + 1];
            const float dx = (px2 - p1.x) * 0.004f, dy = (py2 - p1.y) * 0.004f;
            const float tc = rx * dx + ry * dy, perp = fabsf(rx * dy - ry * dx);
            if (perp > R || tc < -R || (tc - R) > 250.0f * bi) continue;
            // separating axis along the ray normal: the box must straddle the ray line (+2 cm guard)
            if (perp > hx * fabsf(q.c * dy - q.s * dx) + hy * fabsf(q.s * dy + q.c * dx) + 0.02f) continue;
            CNT(c_ex);
            const V2 l2 = rmulT(q, V(p2s[2 * i] - wa.x, p2s[2 * i + 1] - wa.y));
            const V2 dd = vsub(l2, l1);
            float lower = 0.0f, upper = 1.0f; int index = -1; bool ok = true;
            const float num[4] = {n0, n1, n2, n3};
            const float den[4] = {0.0f * dd.x + (-1.0f) * dd.y, 1.0f * dd.x + 0.0f * dd.y, 0.0f * dd.x + 1.0f * dd.y,
                                  (-1.0f) * dd.x + 0.0f * dd.y};
#pragma unroll
            for (int f = 0; f < 4; ++f) {
              if (!ok) break;
              if (den[f] == 0.0f) { if (num[f] < 0.0f) ok = false; }
              else if (den[f] < 0.0f && num[f] < lower * den[f]) { lower = fdiv_cr(num[f], den[f]); index = f; }
              else if (den[f] > 0.0f && num[f] < upper * den[f]) { upper = fdiv_cr(num[f], den[f]); }
              if (upper < lower) ok = false;
            }
            if (ok && index >= 0 && lower < bi) atomicMin(&best[i], __float_as_uint(lower));
          }
        }
      }
#ifdef NASCAR_PROFILE
      if (pass == 0) { PCOUNT(0, c_vis); PCOUNT(1, c_rng); PCOUNT(2, c_open); PCOUNT(3, c_walls); PCOUNT(4, c_wr); PCOUNT(5, c_ex); PCOUNT(6, 1); }
#endif
    }
    if (pass == 0) PROFS(4);
    __syncthreads();   // all lanes of the car are done with best[]
    if (pass == 0) PROFS(5);
    if (active) {
#pragma unroll
      for (int q = 0; q < RPL; ++q) {
        const int i = r * RPL + q;
        const float val = sensor_value(__uint_as_float(best[i]));
        if (pass == 0) {
          if (mode & PM_A_OBS) obs[(size_t)n * 38 + 22 + i] = val;
          if (mode & PM_A_TERM) terminal_obs[(size_t)n * 38 + 22 + i] = val;
        } else {
          obs[(size_t)n * 38 + 22 + i] = val;
        }
      }
    }
    if (pass == 0) PROFS(6);
    if (pass == 0) PROFS_RT(15);
    if (!__syncthreads_or(mode & PM_B_OBS)) break;   // barrier: best / p2 are reused by pass 1
  }
#undef SW_A
#undef SW_B
#undef SW_G
}

// ------------------------------------------------------------------ ray_sensor_kernel: one lane per ray
#ifndef WALL_CAST_SELECT
#define WALL_CAST_SELECT 1   // face loop as selects: 166.6 -> 161.4 us/step sharded (VALU-bound walks, fewer divergent branches)
#endif
// b2PolygonShape::RayCast of one wall box for the ray p1 -> p2 (the arithmetic of sensor_kernel's inner
// loop: same culls, same face order and f32 operations); returns min(bi, hit fraction).
// (dx, dy): the ray direction, cull only.
__device__ __forceinline__ float wall_cast(const float4 wa, const float4 wb, V2 p1, float p2x, float p2y, float dx,
                                           float dy, float bi) {
  const float rx = wa.x - p1.x, ry = wa.y - p1.y;
  const float R = wa.z;
  const float tc = rx * dx + ry * dy, perp = fabsf(rx * dy - ry * dx);
  if (perp > R || tc < -R || (tc - R) > 250.0f * bi) return bi;
  Rot q; q.s = wb.x; q.c = wb.y;
  const float hx = wa.w, hy = wb.z;
  if (perp > hx * fabsf(q.c * dy - q.s * dx) + hy * fabsf(q.s * dy + q.c * dx) + 0.02f) return bi;
  const V2 l1 = rmulT(q, V(p1.x - wa.x, p1.y - wa.y));
  // Box2D's num_f = dot(normal_f, vertex_f - l1) and den_f = dot(normal_f, d) with the box normals (0, -1), (1, 0),
  // (0, 1), (-1, 0): the products by 0 and +-1 are dropped.  The values are the same floats except possibly the sign
  // of a zero (0 * x + (-y) vs -y), and a zero's sign never reaches the result: den is only compared (== < > 0, a
  // zero den selects the parallel case), and a zero num can neither lower `lower` (0 < lower * den <= 0 is false
  // for den < 0) nor reach the returned fraction through `upper` (only compared)
  const float n0 = l1.y - (-hy);
  const float n1 = hx - l1.x;
  const float n2 = hy - l1.y;
  const float n3 = l1.x - (-hx);
  const V2 l2 = rmulT(q, V(p2x - wa.x, p2y - wa.y));
  const V2 dd = vsub(l2, l1);
  float lower = 0.0f, upper = 1.0f; int index = -1; bool ok = true;
  const float num[4] = {n0, n1, n2, n3};
  const float den[4] = {-dd.y, dd.x, dd.y, -dd.x};
#if WALL_CAST_SELECT
  // the same face loop as selects (no divergent branches): every face's quotient is computed and applied only
  // where the branchy loop would have assigned it; a face after the loop's break (ok false) changes nothing
#pragma unroll
  for (int f = 0; f < 4; ++f) {
    const float n = num[f], d = den[f];
    const float q = fdiv_cr(n, d);              // unused when d == 0
    const bool z = d == 0.0f;
    const bool lo = !z && d < 0.0f && n < lower * d;
    const bool up = !z && !lo && d > 0.0f && n < upper * d;
    const bool kill = z && n < 0.0f;
    lower = ok && lo ? q : lower;
    index = ok && lo ? f : index;
    upper = ok && up ? q : upper;
    ok = ok && !kill && !(upper < lower);
  }
#else
#pragma unroll
  for (int f = 0; f < 4; ++f) {
    if (!ok) break;
    if (den[f] == 0.0f) { if (num[f] < 0.0f) ok = false; }
    else if (den[f] < 0.0f && num[f] < lower * den[f]) { lower = fdiv_cr(num[f], den[f]); index = f; }
    else if (den[f] > 0.0f && num[f] < upper * den[f]) { upper = fdiv_cr(num[f], den[f]); }
    if (upper < lower) ok = false;
  }
#endif
  return (ok && index >= 0 && lower < bi) ? lower : bi;
}

// One ray without a beam list (car outside the cells build_beams covers): the sensor grid's wall groups
// of the car's cell (all groups outside the grid), culled by range, by whether this ray is in the
// group's angular mask and by the best hit so far, then wall_cast per wall.
__device__ inline float ray_fallback(const TrackDev& T, V2 p1, float p2x, float p2y, float dx, float dy,
                                           float angf, int i) {
  int beg = 0, end = T.ngroup;
  const uint16_t* list = nullptr;
  if (grid_list(T.sn, p1.x, p1.y, beg, end)) list = T.sn.idx;
  else { beg = 0; end = T.ngroup; }
  const float4* __restrict__ sw = T.swall;
  float bi = 2.0f;
  for (int kk = beg; kk < end; ++kk) {
    const float4 G = ldg(T.groups + (list ? (int)ldg(list + kk) : kk));
    const float grx = G.x - p1.x, gry = G.y - p1.y;
    const float d2 = grx * grx + gry * gry;
    if (d2 > (250.0f + G.z) * (250.0f + G.z)) continue;
    const float d = __builtin_amdgcn_sqrtf(d2);
    unsigned mask;
    float dlo;
    if (G.z > 24.0f) {
      const int j = __float_as_int(G.w) & 0xFFFF;
      const float4 wa = ldg(sw + 2 * j), wb = ldg(sw + 2 * j + 1);
      const float ex = wa.w * wb.y, ey = wa.w * wb.x;
      const float cx = wa.x - p1.x, cy = wa.y - p1.y;
      float dseg;
      mask = seg_ray_mask(cx - ex, cy - ey, cx + ex, cy + ey, wb.z * 1.4143f + 0.3f, angf, dseg);
      dlo = (dseg - (wb.z * 1.4143f + 0.3f)) * (1.0f / 250.0f) - 1e-4f;
    } else {
      mask = ray_mask(grx, gry, d, G.z, angf);
      dlo = (d - G.z) * (1.0f / 250.0f) - 1e-4f;
    }
    if (!((mask >> i) & 1u) || dlo > bi) continue;
    const int first = __float_as_int(G.w) & 0xFFFF, cnt = __float_as_int(G.w) >> 16;
    for (int j = first; j < first + cnt; ++j) bi = wall_cast(ldg(sw + 2 * j), ldg(sw + 2 * j + 1), p1, p2x, p2y, dx, dy, bi);
  }
  return bi;
}

// 4x4 transpose inside each quad of lanes (DPP quad_perm, no LDS): lane r holds v[q] = ray r + 4q on entry
// and o[j] = ray 4r + j on exit, so each lane owns 16 contiguous bytes of the car's obs[22:38].
template <int S> __device__ __forceinline__ float quad_rot(float x) {   // lane r of a quad reads lane (r + S) & 3
  constexpr int ctrl = (S & 3) | (((1 + S) & 3) << 2) | (((2 + S) & 3) << 4) | (((3 + S) & 3) << 6);
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), ctrl, 0xF, 0xF, false));
}
__device__ __forceinline__ float sel4(const float v[4], int k) { return k == 0 ? v[0] : k == 1 ? v[1] : k == 2 ? v[2] : v[3]; }
__device__ __forceinline__ void put4(float o[4], int k, float x) {
#pragma unroll
  for (int j = 0; j < 4; ++j) o[j] = k == j ? x : o[j];
}
__device__ __forceinline__ void quad_transpose(const float v[4], float o[4], int r) {
  o[0] = o[1] = o[2] = o[3] = 0.0f;
  put4(o, r, sel4(v, r));
  put4(o, (r + 1) & 3, quad_rot<1>(sel4(v, (r - 1) & 3)));
  put4(o, (r + 2) & 3, quad_rot<2>(sel4(v, (r - 2) & 3)));
  put4(o, (r + 3) & 3, quad_rot<3>(sel4(v, (r - 3) & 3)));
}

// DistanceSensor.get_sensor_distances (src/distance_sensor.py:71-117) on beam lists, 4 lanes per car
// (rays r, r + 4, r + 8, r + 12 on lane r), BLOCK / 4 cars per workgroup, the track's wall image staged in
// LDS.  Passes and modes as sensor_kernel (pose[n]: pass A, pose[N + n]: pass B for auto-reset cars).
// The 16 values of a car are transposed inside its lane quad and stored as 4 x 16 contiguous bytes.
#ifndef RSENSOR_WPE
#define RSENSOR_WPE 6   // 4 lanes per car at 6 waves/SIMD: 41.5 us (8 lanes 53.7, 2 lanes 44.3; 16 lanes 62.4)
#endif
#define RAY_LPC 4     // lanes per car; each lane walks the lists of rays r, r + 4, r + 8, r + 12
#ifndef RAY_HEADS_AHEAD
#define RAY_HEADS_AHEAD 0
#endif
#ifndef RAY_NO_WALK
#define RAY_NO_WALK 0
#endif
// One ray's walk of its beam list (list index li, head record h = G.head[li]): the first BEAM_HEAD entries from
// the head, the rest of the list only when all of them were walked; stops at the first entry whose distance
// bound lies beyond the best hit.  Returns the best b2PolygonShape::RayCast fraction (2 = no hit).
// GW: the wall image sw is the track's global one (read through the L2), else the workgroup's LDS copy.
// A list's continuation from ent[] index k on, walked by this lane alone: RAY_CHUNK entries requested together, walked
// in order to the sentinel or to the first bound beyond the best hit.
template <bool GW>
__device__ __forceinline__ float ray_walk_rest(const BeamGrid& G, const float4* __restrict__ sw, uint32_t k, float bi, V2 p1,
                                               V2 p2, float dx, float dy) {
  for (;; k += RAY_CHUNK) {
    uint32_t v4[RAY_CHUNK];
#pragma unroll
    for (int q = 0; q < RAY_CHUNK; ++q) v4[q] = ldg(G.ent + k + q);
    bool stop = false;
#pragma unroll
    for (int q = 0; q < RAY_CHUNK; ++q) {
      const uint32_t v = v4[q];
      if (beam_beyond(G, v, bi)) { stop = true; break; }
      const int j = beam_wall(G, v);
      PCOUNT(10, 1);
      bi = GW ? wall_cast(ldg(sw + 2 * j), ldg(sw + 2 * j + 1), p1, p2.x, p2.y, dx, dy, bi)
             : wall_cast(sw[2 * j], sw[2 * j + 1], p1, p2.x, p2.y, dx, dy, bi);
    }
    if (stop) break;
  }
  return bi;
}
// COOP: only the head is walked here; *kc gets the continuation's ent[] index when the walk goes on (0: done), for
// ray_walk_coop
template <bool GW, bool COOP = false>
__device__ __forceinline__ float ray_walk(const BeamGrid& G, const float4* __restrict__ sw, int li, const BeamHead& h, V2 p1,
                                          V2 p2, float dx, float dy, uint32_t* kc = nullptr) {
  float bi = 2.0f;
  const uint32_t hv[BEAM_HEAD] = {h.w.x & 0xFFFFu, h.w.x >> 16, h.w.y & 0xFFFFu};
  bool more = true;
#pragma unroll
  for (int k = 0; k < BEAM_HEAD; ++k) {
    const uint32_t v = hv[k];
    if (beam_beyond(G, v, bi)) { more = false; break; }
    const int j = beam_wall(G, v);
    PCOUNT(10, 1);
    bi = GW ? wall_cast(ldg(sw + 2 * j), ldg(sw + 2 * j + 1), p1, p2.x, p2.y, dx, dy, bi)
               : wall_cast(sw[2 * j], sw[2 * j + 1], p1, p2.x, p2.y, dx, dy, bi);
  }
  const uint32_t off = h.w.y >> 16;
  const uint32_t tail = off ? h.cb + off - 1u : 0u;   // (ent[0] is a sentinel: a continuation never starts at 0)
  if (COOP) { *kc = more ? tail : 0u; return bi; }
  if (more && tail != 0u) bi = ray_walk_rest<GW>(G, sw, tail, bi, p1, p2, dx, dy);
  return bi;
}
// The list continuations of a whole wave's rays, walked by the whole wave (one ray per lane, every lane active): per
// round the rays still walking (k != 0) share the 64 lanes, E = 64 / 2^ceil(log2 n) lanes each, and every lane casts
// one entry of its ray's next E entries.  The entries past a list's sentinel (or past the array, padded by
// BEAM_COOP_PAD sentinels) are skipped; a ray is done once its round met the sentinel or a bound beyond its new best.
// Casting entries the sequential walk would not reach changes nothing: their bounds exceed the best hit (the margin
// the sequential stop test uses), so wall_cast's min keeps the same value; results are those of ray_walk, bit for bit.
// A wave's continuation then costs a few rounds instead of its longest list's entries one after another.
#define BEAM_COOP_PAD 64
#ifndef RAY_COOP_WALK
#define RAY_COOP_WALK 1
#endif
// rounds of the cooperative walk before a ray still walking finishes on its own lane (ray_walk_rest).  No bundled
// track's lists come near it; a tools build with a cap of 1 (build(): tools/build/libnascar_coop1.so) sends every long
// walk down that path, and tests/test_gpu_sensors.py checks its values against the product build's
#ifndef RAY_COOP_ROUNDS
#define RAY_COOP_ROUNDS 1024
#endif
// lanes per walking ray and round at most 64 >> RAY_COOP_LGMIN (0: up to the whole wave for a lone ray; 2: 16 lanes, 32
// bytes of 16-bit entries per round -- fewer line fills past a short list's sentinel; DESIGN round-6 table)
#ifndef RAY_COOP_LGMIN
#define RAY_COOP_LGMIN 2
#endif
template <bool GW>
__device__ __forceinline__ float ray_walk_coop(const BeamGrid& G, const float4* __restrict__ sw, uint32_t k, float bi, V2 p1,
                                               V2 p2, float dx, float dy) {
  const int lane = __lane_id();
  const unsigned long long below = lane ? (~0ull >> (64 - lane)) : 0ull;
  for (int round = 0; round < RAY_COOP_ROUNDS; ++round) {   // (a finite list ends every walk; past the cap, see below)
    const unsigned long long m = __ballot(k != 0u);
    if (!m) break;
    const int na = __popcll(m);
    const int lg = max(na > 1 ? 32 - __clz(na - 1) : 0, RAY_COOP_LGMIN);   // ceil(log2 na), at least the minimum
    const int E = 64 >> lg;                               // lanes per walking ray
    const int q = lane >> (6 - lg), o = lane & (E - 1);   // this lane's ray (q-th walking one) and entry offset
    const bool serve = q < na;
    int owner = 0;
    {   // the q-th set bit of m (binary search on popcounts)
      unsigned long long mm = m; int qq = q;
#pragma unroll
      for (int sh = 32; sh >= 1; sh >>= 1) {
        const int c = __popcll(mm & ((1ull << sh) - 1ull));
        if (qq >= c) { qq -= c; mm >>= sh; owner += sh; }
      }
      if (!serve) owner = lane;
    }
    const uint32_t ko = __shfl(k, owner);
    const float bo = __shfl(bi, owner);
    const V2 po = V(__shfl(p1.x, owner), __shfl(p1.y, owner)), qo = V(__shfl(p2.x, owner), __shfl(p2.y, owner));
    const float dxo = __shfl(dx, owner), dyo = __shfl(dy, owner);
    const uint32_t v = serve ? (uint32_t)ldg(G.ent + ko + o) : BEAM_PAD;
    const unsigned long long pm = __ballot(v == BEAM_PAD);
    const unsigned long long gm = (lg == 0 ? ~0ull : ((1ull << E) - 1ull)) << (q * E & 63);
    const bool valid = serve && v != BEAM_PAD && !(pm & gm & below);
    float c = bo;
    if (valid) {
      const int j = beam_wall(G, v);
      PCOUNT(10, 1);
      c = GW ? wall_cast(ldg(sw + 2 * j), ldg(sw + 2 * j + 1), po, qo.x, qo.y, dxo, dyo, bo)
             : wall_cast(sw[2 * j], sw[2 * j + 1], po, qo.x, qo.y, dxo, dyo, bo);
    }
    for (int sh = 1; sh < E; sh <<= 1) c = fminf(c, __shfl_xor(c, sh));   // the group's best (min over its lanes)
    // this lane's own ray: its group's best, sentinel, and the bound of the group's last entry
    const int qm = __popcll(m & below);                  // rank of this lane's ray among the walking ones
    const int g0 = (qm * E) & 63;
    const float gb = __shfl(c, g0);
    const uint32_t vl = __shfl(v, g0 + E - 1);
    const unsigned long long gmo = (lg == 0 ? ~0ull : ((1ull << E) - 1ull)) << g0;
    if (k != 0u) {
      bi = gb;
      const bool stop = (pm & gmo) != 0ull || beam_beyond(G, vl, bi);
      k = stop ? 0u : k + (uint32_t)E;
    }
  }
  if (k != 0u) bi = ray_walk_rest<GW>(G, sw, k, bi, p1, p2, dx, dy);   // (product build: lists of thousands of entries)
  return bi;
}
__device__ __forceinline__ int beam_slot0(double ang) {   // list slot of ray 0's direction bin (see ray_lane)
  double u = ang * (BEAM_NB / (2.0 * PI_D));
  u -= BEAM_NB * floor(u * (1.0 / BEAM_NB));
  return beam_slot(min(BEAM_NB - 1, max(0, (int)u)));
}

// The 4-lane work of car n, lane r (rays r, r + 4, r + 8, r + 12) in ray_sensor_kernel / rollout_kernel: both
// passes, the beam-list walks against the wall image sw (LDS), the quad transpose and the obs stores.
// All 4 lanes of a car are consecutive lanes of one quad and call this together.
// LPC = 16 (small batches, see launch_sensors_impl): one ray per lane, the 16 lanes of a car store its 16 values
// directly (64 contiguous bytes per car).
// COOP: the wave-cooperative list continuations when every lane of the wave is here (16 lanes per car); false: every
// ray walks its own list (callers whose lanes are not lockstep rays of whole cars, e.g. rt_switch_kernel)
template <int LPC = RAY_LPC, bool GW = false, bool COOP = true>
__device__ __forceinline__ void ray_lane(const Params& P, const TrackDev& T, const float4* __restrict__ sw, int n, int r,
                                         float* obs, float* terminal_obs, int passes) {
  static_assert(LPC == 4 || LPC == 16, "lanes per car");
  constexpr int RPL = 16 / LPC;
  // pose loads after the staging barrier: issuing them (and pass A's cos/sin) before it, or the beam-cell
  // lookup too, measured 2.5 / 9 us slower (registers held across the staging)
  // each pass loads its own pose (pass B's only for auto-reset cars): no pose is held across the other pass's
  // walks (held, both had been spilled to scratch at 80 VGPRs); pass B's mode word is read up front
  // one ray per lane: its offset's cos / sin requested first, beside the pose loads (not behind the cell lookup)
  const double2 rk = LPC == 16 ? ldg((const double2*)P.ray_cs + r) : make_double2(0.0, 0.0);
  int mode = 0;
  // a step's passes (A and B) read pass B's record only for this step's auto-reset envs (Params::reset_env); a pass-B-only
  // call (rt_switch_kernel, the rollout's pass-B loop) names cars whose record it has just written
  if ((passes & 2) && (!(passes & 1) || P.reset_env[(unsigned)n / (unsigned)P.C])) mode = __float_as_int(P.pose[P.N + n].w) & PM_B_OBS;
  const BeamGrid G = T.beam;
#pragma unroll 1
  for (int pass = 0; pass < 2; ++pass) {
    if (pass == 0 && !(passes & 1)) continue;
    if (pass == 1 && !(mode & PM_B_OBS)) continue;
    const float4 ps = P.pose[pass == 0 ? (size_t)n : (size_t)P.N + n];
    if (pass == 0) mode |= __float_as_int(ps.w) & (PM_A_OBS | PM_A_TERM);
    if (pass == 0 && !(mode & (PM_A_OBS | PM_A_TERM))) continue;
    const V2 p1 = V(ps.x, ps.y);
    const double px = ps.x, py = ps.y, ang = ps.z;
    const double2 cs = P.pose_cs[pass == 0 ? (size_t)n : (size_t)P.N + n];
    if (LPC == 16 && pass == 0) PROFR(2);   // profile builds (16 lanes per car): pose loaded
    const int2 cell = beam_cell(G, p1.x, p1.y);
    const int base = cell.x;
    if (LPC == 16 && pass == 0) { asm volatile("" :: "v"(base)); PROFR(3); }   // beam cell looked up
    // direction bin of sa = -radians(22.5 i) + ang (f64; the lists carry a 2e-3 rad guard) -> list slot
    // ray i is exactly BEAM_STRIDE bins clockwise of ray 0 in real arithmetic, and the f64 rounding of
    // sa_i (~1e-15 rad) is far inside the lists' 2e-3 rad guard, so bin_i = bin_0 - BEAM_STRIDE i:
    // slot_i = (bin_0 % STRIDE) * 16 + (bin_0 / STRIDE - i) mod 16
    int slot0;
    {
      double u = ang * (BEAM_NB / (2.0 * PI_D));
      u -= BEAM_NB * floor(u * (1.0 / BEAM_NB));
      slot0 = beam_slot(min(BEAM_NB - 1, max(0, (int)u)));
    }
    auto slot_of = [&](int i) { return (slot0 & ~15) | ((slot0 - i) & 15); };
    float v[RPL];
#pragma unroll
    for (int q = 0; q < RPL; ++q) v[q] = 0.0f;
#if RAY_HEADS_AHEAD
    // the four rays' list heads requested together (independent 8-byte loads) before the first walk
    BeamHead hd[RPL];
#pragma unroll
    for (int q = 0; q < RPL; ++q) {
      if (base >= 0) hd[q] = beam_head(G, cell, base + slot_of(r + LPC * q));
      else hd[q] = BeamHead{make_uint2(0u, 0u), 0u};
    }
#pragma unroll
#else
#pragma unroll 1
#endif
    for (int q = 0; q < RPL; ++q) {
      const int i = r + LPC * q;
      double dxd, dyd;
      float fx = ps.x, fy = ps.y, fa = ps.z;   // widened per ray: three floats live across the walks, not three doubles
      asm volatile("" : "+v"(fx), "+v"(fy), "+v"(fa));
      const V2 p2 = LPC == 16 ? ray_end_k((double)fx, (double)fy, (double)fa, cs.x, cs.y, i, rk, dxd, dyd)
                              : ray_end(P, (double)fx, (double)fy, (double)fa, cs.x, cs.y, i, dxd, dyd);
      const float dx = (p2.x - p1.x) * 0.004f, dy = (p2.y - p1.y) * 0.004f;   // cull only
      float bi = 2.0f;
      uint32_t kc = 0u;   // (wave-cooperative continuation: this ray's next ent[] index, 0 when its walk is done)
      const bool coop = COOP && LPC == 16 && RAY_COOP_WALK && __ballot(1) == ~0ull;   // every lane active: wave-uniform
      if (base >= 0) {
        const int sl = slot_of(i);
#if RAY_HEADS_AHEAD
        bi = ray_walk<GW>(G, sw, base + sl, hd[q], p1, p2, dx, dy);
#elif RAY_NO_WALK   // timing probe only (wrong results): the head load without the walk
        const BeamHead h = beam_head(G, cell, base + sl);
        bi = __uint_as_float((h.w.x & 1u) | 0x3f800000u);
#else
#ifdef NASCAR_PROFILE
        const BeamHead hh = beam_head(G, cell, base + sl);
        if (LPC == 16 && pass == 0) { PROFR(4); asm volatile("" :: "v"(hh.w.x)); PROFR(5); }   // end points; head loaded
        if (LPC == 16 && coop) bi = ray_walk<GW, true>(G, sw, base + sl, hh, p1, p2, dx, dy, &kc);
        else bi = ray_walk<GW>(G, sw, base + sl, hh, p1, p2, dx, dy);
#else
        if (LPC == 16 && coop) bi = ray_walk<GW, true>(G, sw, base + sl, beam_head(G, cell, base + sl), p1, p2, dx, dy, &kc);
        else bi = ray_walk<GW>(G, sw, base + sl, beam_head(G, cell, base + sl), p1, p2, dx, dy);
#endif
#endif
      } else {
        PCOUNT(9, 1);
        bi = ray_fallback(T, p1, p2.x, p2.y, dx, dy, ps.z, i);
      }
      if (LPC == 16 && coop) bi = ray_walk_coop<GW>(G, sw, kc, bi, p1, p2, dx, dy);   // (wave-uniform branch)
      PCOUNT(8, 1);
      if constexpr (RPL == 4) put4(v, q, sensor_value(bi));
      else v[q] = sensor_value(bi);
    }
    // lane index and car index made opaque here, so the transpose indices and the store addresses derived from
    // them are computed now rather than held (spilled) across the walks
    int rq = r, nq = n;
    asm volatile("" : "+v"(rq), "+v"(nq));
    if constexpr (RPL == 4) {
      float o[4];
      quad_transpose(v, o, rq);
      const size_t at = (size_t)nq * 38 + 22 + 4 * rq;   // 8-byte aligned (rows are 152 B)
      const float2 lo = make_float2(o[0], o[1]), hi = make_float2(o[2], o[3]);
      if (pass == 1 || (mode & PM_A_OBS)) { *(float2*)(obs + at) = lo; *(float2*)(obs + at + 2) = hi; }
      if (pass == 0 && (mode & PM_A_TERM)) { *(float2*)(terminal_obs + at) = lo; *(float2*)(terminal_obs + at + 2) = hi; }
    } else {
      if (pass == 0) { asm volatile("" :: "v"(v[0])); PROFR(6); }   // profile builds: walk done
      const size_t at = (size_t)nq * 38 + 22 + rq;
      if (pass == 1 || (mode & PM_A_OBS)) obs[at] = v[0];
      if (pass == 0 && (mode & PM_A_TERM)) terminal_obs[at] = v[0];
    }
  }
}

// rollout_kernel's sensor phase for one block: thread t owns lane r = t % 4 of the cars in slots t / 4 + 32 j
// (j = 0..3, RAY_LPC rounds of ray_lane's mapping).  At the fused kernel's low occupancy the dependent loads
// of a lane (pose -> beam cell -> list heads) are not hidden by other waves, so they are issued for all four
// cars and all 16 of the thread's rays at once before any list is walked.  Pass B (auto-reset cars) goes
// through ray_lane per car.  Same walks and results as ray_lane.
__device__ __forceinline__ void ray_block_batched(const Params& P, const TrackDev& T, const float4* __restrict__ sw,
                                                  float* obs, int passes) {
  static_assert(RAY_LPC == 4, "batched sensor mapping");
  constexpr int CPR = SBLOCK / RAY_LPC;   // cars per round: NJ rounds cover the block's SBLOCK slots
  constexpr int NJ = 4, RPL = 4;
  const int t = threadIdx.x, r = t & 3, C = P.C;
  const BeamGrid G = T.beam;
  int n[NJ], slot0[NJ];
  int2 base[NJ];   // beam cell records (list base, first ent[] index)
  bool ok[NJ];
  float4 pa[NJ];
  double2 cs[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int lc = (t >> 2) + CPR * j, el = lc / C, car = lc - el * C;
    const int env = blk_env_of(P, el, blockIdx.x * P.epb + el);
    ok[j] = env >= 0;
    n[j] = ok[j] ? env * C + car : 0;
  }
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    pa[j] = ok[j] ? P.pose[n[j]] : make_float4(0.f, 0.f, 0.f, 0.f);
    cs[j] = ok[j] ? P.pose_cs[n[j]] : make_double2(1.0, 0.0);
  }
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    ok[j] = ok[j] && (__float_as_int(pa[j].w) & PM_A_OBS) != 0;
    base[j] = ok[j] ? beam_cell(G, pa[j].x, pa[j].y) : make_int2(-1, 0);
    slot0[j] = beam_slot0((double)pa[j].z);
  }
  V2 p2[NJ][RPL];
  BeamHead hd[NJ][RPL];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
#pragma unroll
    for (int q = 0; q < RPL; ++q) {
      double dxd, dyd;
      p2[j][q] = ray_end(P, pa[j].x, pa[j].y, pa[j].z, cs[j].x, cs[j].y, r + RAY_LPC * q, dxd, dyd);
      const int sl = (slot0[j] & ~15) | ((slot0[j] - (r + RAY_LPC * q)) & 15);
      if (base[j].x >= 0) hd[j][q] = beam_head(G, base[j], base[j].x + sl);
      else hd[j][q] = BeamHead{make_uint2(0u, 0u), 0u};
    }
  }
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    if (!ok[j]) continue;                    // uniform over the car's quad
    const V2 p1 = V(pa[j].x, pa[j].y);
    float v[RPL] = {0.0f, 0.0f, 0.0f, 0.0f};
    // the car's four heads / end points as named values rotated one place per ray (a select on the ray index
    // became a dynamically indexed array in scratch memory)
    BeamHead h0 = hd[j][0], h1 = hd[j][1], h2 = hd[j][2], h3 = hd[j][3];
    V2 e0 = p2[j][0], e1 = p2[j][1], e2 = p2[j][2], e3 = p2[j][3];
#pragma unroll 1
    for (int q = 0; q < RPL; ++q) {
      const int i = r + RAY_LPC * q;
      const V2 e = e0;
      const float dx = (e.x - p1.x) * 0.004f, dy = (e.y - p1.y) * 0.004f;   // cull only
      float bi;
      if (base[j].x >= 0) {
        const int sl = (slot0[j] & ~15) | ((slot0[j] - i) & 15);
        bi = ray_walk<false>(G, sw, base[j].x + sl, h0, p1, e, dx, dy);
      } else {
        bi = ray_fallback(T, p1, e.x, e.y, dx, dy, pa[j].z, i);
      }
      put4(v, q, sensor_value(bi));
      h0 = h1; h1 = h2; h2 = h3; e0 = e1; e1 = e2; e2 = e3;
    }
    float o[4];
    quad_transpose(v, o, r);
    const size_t at = (size_t)n[j] * 38 + 22 + 4 * r;
    *(float2*)(obs + at) = make_float2(o[0], o[1]); *(float2*)(obs + at + 2) = make_float2(o[2], o[3]);
  }
  if (passes & 2) {
#pragma unroll 1
    for (int j = 0; j < NJ; ++j) {
      const int lc = (t >> 2) + CPR * j, el = lc / C, car = lc - el * C;
      const int env = blk_env_of(P, el, blockIdx.x * P.epb + el);
      if (env >= 0 && P.reset_env[env]) ray_lane(P, T, sw, env * C + car, r, obs, nullptr, 2);
    }
  }
}
// LPC lanes per car, BLOCK / LPC cars per workgroup; `sub` sensor workgroups per step-kernel workgroup (enough for
// its epb * C cars)
template <int LPC, int RB = BLOCK, bool GW = false>
__global__ void __launch_bounds__(RB) __attribute__((amdgpu_waves_per_eu(RSENSOR_WPE)))
ray_sensor_kernel(Params P, float* obs, float* terminal_obs, int passes, int SUB) {
  constexpr int CPW = RB / LPC;
  const int bx = blockIdx.x, b = bx / SUB + P.blk0, sub = bx % SUB;
  const int t = threadIdx.x, lc = t / LPC, r = t - lc * LPC;
  const int C = P.C;
  const int slot = sub * CPW + lc;
  const int el = slot / C, car = slot - el * C;
  const int env = blk_env_of(P, el, b * P.epb + el);
  if (blk_empty(P, b)) return;   // an empty workgroup of a device-built block map (random-track mode)
  const TrackDev& T = P.tracks[blk_track_of(P, b)];
  PROF_B0(P.blk0 * SUB);   // profile builds: stamp rows numbered over the whole grid (the sharded rollout's shards)
  PROFR_RT(14); PROFR(0); PROFR_XCC(8);   // profile builds: stamp slots 0-7 (16 lanes per car: ray_lane's 2-6), realtime 14 / 15
  if constexpr (GW) {   // walls read from the track's global image: no staging, no LDS, no barrier
    PROFR(1);
    if (env < 0) return;
    ray_lane<LPC, true>(P, T, T.swall, env * C + car, r, obs, terminal_obs, passes);
    PROFR(7); PROFR_RT(15);
    return;
  }
  {
    float4* s_w = (float4*)smem;
    const int nw2 = 2 * T.nwall;
    for (int k = t; k < nw2; k += RB) s_w[k] = ldg(T.swall + k);
    __syncthreads();
  }
  PROFR(1);
  if (env < 0) return;
  ray_lane<LPC>(P, T, (const float4*)smem, env * C + car, r, obs, terminal_obs, passes);
  PROFR(7); PROFR_RT(15);
}

__device__ __forceinline__ uint32_t mix32(uint64_t x) {   // splitmix64 finaliser
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  x ^= x >> 31;
  return (uint32_t)(x >> 32);
}
// Noisy rule driver (policy 3): with probability NOISE_P16 / 65536 per car-step the driver's action is
// replaced by the uniform draw of policy 0 (the driver state still advances), as gen_golden.py's
// "rule_noisy" mode does with a host RNG; cars of one env therefore leave the common start trajectory.
#define NOISE_P16 9830u   // 0.15 * 65536
// device action sources 0, 1, 3 for car n from its current observation row (policy 2, the SAC actor, is
// actor_kernel): writes (throttle_brake, steering) to a0, a1
__device__ __forceinline__ void policy_car(int policy, uint64_t seed, int64_t step, int n, const float* obs, double* ctl,
                                           float& a0, float& a1) {
  const uint64_t key = (seed * 0x100000001B3ull) ^ ((uint64_t)n << 24) ^ (uint64_t)step * 0x9E3779B1ull;
  const float u0 = (float)(mix32(key) >> 8) * (2.0f / 16777216.0f) - 1.0f;
  const float u1 = (float)(mix32(key ^ 0xABCDEF12345ull) >> 8) * (2.0f / 16777216.0f) - 1.0f;
  if (policy == 0) { a0 = u0; a1 = u1; return; }
  // BaseController._fallback_control (game/control/base_controller.py:39-103); state per car in ctl[4*n..]:
  // throttle_brake is a Python float (float64 += 0.1, *= 0.5, clamps); steering, speed_limit and
  // last_forward hold numpy float32 values (NEP 50: float32 op python scalar stays float32).
  const float* o = obs + (size_t)n * 38;
  double* s = ctl + 4 * (size_t)n;   // throttle_brake, steering, last_forward, speed_limit
  const float fwd = o[22], spd = o[4];
  float steer = (float)s[1], last = (float)s[2], lim = (float)s[3];
  double tb = s[0];
  if (last >= fwd) lim = fwd;
  if (last < fwd) lim = 1.0f;
  if (spd < lim * 0.95f) tb += 0.1;
  if (spd > lim * 1.05f) tb -= 0.1;
  const float r = o[22 + 15], l = o[22 + 1];
  if (r > l) steer = 1.0f - (l / r);
  else if (l > r) steer = (1.0f - (r / l)) * -1.0f;
  else steer *= 0.9f;
  if (fabsf(steer) > 0.25f) tb *= 0.5;
  tb = tb > 1.0 ? 1.0 : tb;  tb = tb < -1.0 ? -1.0 : tb;            // max(min(tb, 1), -1)
  steer = steer > 1.0f ? 1.0f : steer;  steer = steer < -1.0f ? -1.0f : steer;
  s[0] = tb; s[1] = steer; s[2] = fwd; s[3] = lim;
  if (policy == 3 && (mix32(key ^ 0x5DEECE66Dull) >> 16) < NOISE_P16) { a0 = u0; a1 = u1; }
  else { a0 = (float)tb; a1 = steer; }
}
__global__ void policy_kernel(int N, int policy, uint64_t seed, int64_t step, const float* obs, float* act, double* ctl) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  float a0, a1;
  policy_car(policy, seed, step, n, obs, ctl, a0, a1);
  act[2 * n] = a0; act[2 * n + 1] = a1;
}



// CarEnv action -> CarPhysics.step for one car whose physics state is loaded in c (src/car_env.py:733-740,
// src/car_physics.py:341-384): BaseEnv._convert_to_internal_action of (tb, st), Car.update_physics, the
// Box2D step; writes the model / body state back and the sensor pass-A pose.
// logic_ahead (model_logic_kernel): the car's lap-timer / bookkeeping fields are requested right after its Box2D step
__device__ __forceinline__ void model_car(const Params& P, Car& c, int n, const TrackDev& T, float tb, float st, int want_term,
                                          bool logic_ahead = false) {
  const WallSet S{T.walls, T.nwall, T.bp, T.sn, T.wfat, P.ct};
  float a0, a1, a2 = st;
  if (tb >= 0) { a0 = tb; a1 = 0.0f; } else { a0 = 0.0f; a1 = -tb; }
  if (c.disabled) { a0 = 0.0f; a1 = 0.0f; a2 = 0.0f; }
  c.thr_in = pymax(0.0, pymin(1.0, (double)a0));
  c.brk_in = pymax(0.0, pymin(1.0, (double)a1));
  c.str_in = pymax(-1.0, pymin(1.0, (double)a2));
#ifndef NASCAR_KO_UPDATE   // knockout timing builds only (see b2_step)
  car_update_physics(P, c, n, T);
#endif
  car_store_model(P, n, c);
  asm volatile("" ::: "memory");   // keep the model write-back ahead of the Box2D step (register pressure)
  PROF(3);
  b2_step(c, S, P.dt_f, P.friction);
  PROF(4);
  if (logic_ahead) car_load_logic(P, n, c);   // used by the logic half (model_block)
  if (ct_in_lds(c)) {   // model_kernel's LDS records back to the car's global ones (live and dead, see ct_make_room)
    DContact* g = P.ct + (size_t)n * MAXC;
    for (int i = 0; i < c.ct_hw; ++i) g[i] = c.ct[i];
  }
  car_store_body(P, n, c);
  set_pose(P, n, c, PM_A_OBS | (want_term ? PM_A_TERM : 0));   // sensor pass A
}

// The env step as two launches: model_kernel (actions -> Car.update_physics -> Box2D step, one lane
// per car; its TOI code holds it at one wave per SIMD) hands the body / listener state to logic_kernel
// (banking, disable logic, lap timer, rewards, termination, obs, auto-reset) through the state arrays.
#ifndef MODEL_CT_LDS
#define MODEL_CT_LDS 1      // model_kernel holds cars' contact records in LDS (CT_LDS_CAP per lane, dynamic shared memory)
#endif
// a lane's slots padded to an odd number of 16-byte units, so the lanes' same-record accesses spread over the banks
#define CT_LDS_STRIDE ((CT_LDS_CAP * sizeof(DContact) / 16) % 2 ? CT_LDS_CAP * sizeof(DContact) : CT_LDS_CAP * sizeof(DContact) + 16)
#define MODEL_CT_LDS_BYTES (MODEL_CT_LDS ? (size_t)SBLOCK * CT_LDS_STRIDE : (size_t)0)
#ifndef MODEL_WPE
#define MODEL_WPE 2   // 2 waves/SIMD (233 VGPRs, 244 fused with the logic, no spills since the LDS islands; round 1: 1 wave/SIMD
                      // with 256 + 44 AGPRs measured 103.6 vs 100.6 us/step)
#endif
// policy >= 0: the actions come from device action source `policy` (policy_car, nascar_step_driven) on the
// current obs instead of the actions buffer -- the closed-loop driver's step without a policy_kernel launch.
// Every thread of the block calls it (it holds the segment staging barrier); lanes without a car (env < 0) skip
// the step (model_kernel: they return; FUSED, the model_logic_kernel, keeps them for the barriers after it).
// FUSED (model_logic_kernel): the car's lap-timer / bookkeeping fields (car_load_logic) are requested right after its
// Box2D step (held across it they spilled) and kept in c for the logic half, which continues from c (its body fields
// are the ones car_store_body writes) instead of reloading them: the slowest wave's logic half no longer starts with
// a memory round trip.
// the track's segments, staged in LDS by the step kernels' model half (model_logic_kernel's logic half reads them too)
__shared__ DSeg g_step_segs[MAX_SEG];
// one segment's logic tables (chord prefix sum, f32 chord screen), held in registers by lane tid = segment from the
// model half's staging to the logic half's (no global round trip there)
struct SegReg { double prefix; float4 sg; float rll; };
__device__ __forceinline__ void seg_tables(const DSeg& sg, double prefix, SegReg& r) {   // as stage_track_lds
  r.prefix = prefix;
  const double dx = sg.ex - sg.sx, dy = sg.ey - sg.sy, ll = dx * dx + dy * dy;
  r.sg = make_float4((float)sg.sx, (float)sg.sy, (float)dx, (float)dy);
  r.rll = ll < 1e-6 ? 0.0f : (float)(1.0 / ll);
}
template <bool FUSED>
__device__ __forceinline__ void model_block(const Params& P, const void* actions, int discrete, int want_term, int policy,
                                            uint64_t seed, int64_t step, const float* pobs, int tid, int env, int n, Car& c,
                                            SegReg& sr) {
  PROF_B0(P.blk0);   // profile builds: stamp rows numbered over the whole grid (the sharded rollout's shards)
  PROF_RT(14);
  PROF_XCC(10);
  PROF(0);
#if MODEL_PRIO == 1   // A/B: model_kernel's waves issue ahead of co-resident logic / sensor waves of other shards
  __builtin_amdgcn_s_setprio(2);
#endif
  // car state and action requested before the segment staging barrier (their round trips overlap the
  // staging's instead of following it: 89 -> 84 us per step)
  if (env >= 0) car_load_phys(P, n, c);
  c.pid = n;
#if MODEL_CT_LDS
  // the car's contact records into its LDS slots (lists of up to CT_LDS_CAP; longer ones stay global): the
  // loads are issued before the staging barrier, and every b2Contact access of the step is then an LDS one
  if (env >= 0 && c.nct <= CT_LDS_CAP) {
    DContact* s_ct = (DContact*)(smem + (size_t)tid * CT_LDS_STRIDE);
    for (int i = 0; i < c.nct; ++i) s_ct[i] = c.ct[i];
    c.ct = s_ct;
    c.ct_hw = c.nct;
  }
#endif
  // actions (BaseEnv._convert_to_internal_action / _discrete_to_continuous, np.float32)
  float tb = 0.0f, st = 0.0f;
  if (env >= 0 && policy >= 0) {
    policy_car(policy, seed, step, n, pobs, P.ctl, tb, st);
  } else if (env >= 0) {
    if (discrete) {
      int a = ((const int*)actions)[n];
      tb = a == 1 ? 1.0f : (a == 2 ? -1.0f : 0.0f);
      st = a == 3 ? -1.0f : (a == 4 ? 1.0f : 0.0f);
    } else {
      tb = ((const float*)actions)[2 * n]; st = ((const float*)actions)[2 * n + 1];
    }
  }
  TrackDev T = P.tracks[blk_track_of(P, wg_block(P))];
  if (tid < T.nseg) {
    const DSeg sg = ldg(T.segs + tid);
    g_step_segs[tid] = sg;
    if (FUSED) seg_tables(sg, ldg(T.prefix + tid), sr);
  }
  __syncthreads();
  T.segs = g_step_segs;   // (the wall table stays global: staged in LDS it measured neutral, and the LDS holds the contacts)
  PROF(1);
  if (!FUSED && env < 0) return;
  if (env >= 0) {
    PROF(2);
    model_car(P, c, n, T, tb, st, want_term, FUSED);
    PROF(5);
    PROF_RT(15);
  }
}
__global__ void __launch_bounds__(SBLOCK) __attribute__((amdgpu_waves_per_eu(MODEL_WPE))) model_kernel(Params P, const void* actions, int discrete, int want_term,
                                                                                                    int policy, uint64_t seed, int64_t step, const float* pobs) {
  const int tid = threadIdx.x, C = P.C;
  const int el = tid / C, car = tid - el * C;
  const int slot = wg_block(P) * P.epb + el;
  const int env = blk_env_of(P, el, slot);
  if (blk_empty(P, wg_block(P))) return;   // empty workgroup (device-built block map)
  Car c;
  SegReg sr;
  model_block<false>(P, actions, discrete, want_term, policy, seed, step, pobs, tid, env, env >= 0 ? env * C + car : 0, c, sr);
}

// logic_kernel's shared memory: the env passes' per-car words
struct LogicLDS {
  int laps_old[SBLOCK], dis_old[SBLOCK], laps_new[SBLOCK], dis_new[SBLOCK], lapdone[SBLOCK];
  int dis_final[SBLOCK], below[SBLOCK], envdone[SBLOCK];
};
// the block's track segments in LDS (f64 segments, chord prefix sums, f32 chord screens)
struct TrackLDS { DSeg segs[MAX_SEG]; double prefix[MAX_SEG]; float4 sg[MAX_SEG]; float rll[MAX_SEG]; };
__device__ __forceinline__ void stage_track_lds(const TrackDev& T, TrackLDS& TL, int tid) {
  if (tid < T.nseg) {
    const DSeg sg = ldg(T.segs + tid);
    TL.segs[tid] = sg; TL.prefix[tid] = ldg(T.prefix + tid);
    const double dx = sg.ex - sg.sx, dy = sg.ey - sg.sy, ll = dx * dx + dy * dy;
    TL.sg[tid] = make_float4((float)sg.sx, (float)sg.sy, (float)dx, (float)dy);
    TL.rll[tid] = ll < 1e-6 ? 0.0f : (float)(1.0 / ll);
  }
}
// logic state of car n (body from model_kernel, lap timer / bookkeeping, tyres) and its env's time / pending /
// reason words (read by car 0's lane in the env passes)
__device__ __forceinline__ void logic_load_env(const Params& P, int env, int car, double& sim, int& pend_in, int& reason_in) {
  sim = 0.0; pend_in = 0; reason_in = 0;
  if (env >= 0) {
    if (car == 0) {   // reason_in bit 8: the env was never reset (E_CREATED == 0)
      pend_in = P.env_i32[E_PENDING * P.E + env];
      reason_in = P.env_i32[E_REASON * P.E + env] | (P.env_i32[E_CREATED * P.E + env] == 0 ? 0x100 : 0);
    }
    sim = P.env_time[env];
  }
}
__device__ __forceinline__ void logic_load(const Params& P, int env, int car, int n, Car& c, double& sim, int& pend_in,
                                           int& reason_in) {
  if (env >= 0) {
    car_load_body(P, n, c);
    car_load_logic(P, n, c);
    car_reload_tyres(P, n, c);
  }
  logic_load_env(P, env, car, sim, pend_in, reason_in);
}
// model_logic_kernel: the logic half continues from the model half's c (body fields as car_store_body stored them,
// logic fields requested at the start, see model_block), with car_load_body's derived fields and global list pointers
__device__ __forceinline__ void logic_from_model(const Params& P, int n, Car& c) {
  car_reload_tyres(P, n, c);   // (written back before the Box2D step, not held across it)
  if (P.car_contact) {         // car_contact_block rewrote velocities / impulses in the arena: reload the body
    car_load_body(P, n, c);
    return;
  }
  c.just_disabled = 0;
  c.force = zero2(); c.torque = 0.0f; c.c0 = c.c; c.a0 = c.a; c.alpha0 = 0.0f; c.moved = 0;
  c.ct = P.ct + (size_t)n * MAXC; c.act_key = P.act_key + (size_t)n * MAXC; c.act_n = P.act_n + (size_t)n * MAXC * 2;
  c.acc = nullptr;
}
// the rest of the env step for one block (every thread calls it; it holds block barriers): banking, impulse /
// stuck / backward disable, lap timer, env pass 1, obs[0:22], rewards, env pass 2 (termination), auto-reset
// (sensor pass-B pose), state write-back, coalesced obs rows.  T.segs / T.prefix point at TL.
__device__ __forceinline__ void logic_run(const Params& P, const TrackDev& T, const TrackLDS& TL, LogicLDS& L, int tid,
                                          int el, int car, int env, int n, Car& c, double sim, int pend_in, int reason_in,
                                          float* obs, float* reward, uint8_t* car_flags, uint8_t* env_flags, int auto_reset,
                                          float* terminal_obs) {
  const int C = P.C;
  const ChordScreen CS{TL.sg, TL.rll, T.nseg};
  double prog_now = 0.0;   // track_progress at the step's final body position
  const int nw = T.nwall;
  const WallSet S{T.walls, nw, T.bp, T.sn, T.wfat};
  bool lapdone = false;
  if (env >= 0) {
    L.dis_old[tid] = c.disabled;
    LPROF(1);
    L.laps_old[tid] = c.lt_laps;   // the lap count does not change before lap_update
    const uint64_t cand = screen_candidates(CS, c.xf.p.x, c.xf.p.y);   // the body position is final for this step
    // the banking and the track progress (the rewards' _calculate_multi_rewards needs it below) in one chord pass
    if (T.has_banking) c.bank = bank_and_progress_screened(T, cand, c.xf.p.x, c.xf.p.y, prog_now);
    else { c.bank = 0.0; prog_now = track_progress_screened(T, cand, c.xf.p.x, c.xf.p.y); }
    if (!c.disabled) {   // _run_single_physics_step (src/car_env.py:582-638)
      double imp = c.imp_present ? c.imp : 0.0;
      if (imp > 50000.0) { c.disabled = 1; c.just_disabled = 1; }
      if (imp > 100.0) c.cum_impact += imp;
      if (c.cum_impact > 250000.0 && !c.disabled) { c.disabled = 1; c.just_disabled = 1; }
      double speed = (double)vlen(c.v);
      if (speed < 0.5) c.stuck_dur = c.stuck_dur + P.dt_d;
      else { c.stuck_dur = 0.0; c.has_stuck_start = 0; }
    }
    lapdone = lap_update(T, CS, c, c.xf.p.x, c.xf.p.y, sim);
    L.laps_new[tid] = c.lt_laps; L.dis_new[tid] = c.disabled; L.lapdone[tid] = lapdone;
  }
  LPROF(2);
  __syncthreads();
  // env pass 1: lap-reset pending (src/car_env.py:672-676 with _all_active_cars_completed_lap :1640-1669,
  // evaluated in car order with cars > i not yet updated)
  int pend_env = 0;
  if (env >= 0 && car == 0) {
    int pend = pend_in;
    if (P.reset_on_lap) {
      const int b = tid;
      for (int i = 0; i < C; ++i) {
        if (!L.lapdone[b + i]) continue;
        bool any = false, all = true;
        for (int j = 0; j < C; ++j) {
          int dis = j <= i ? L.dis_new[b + j] : L.dis_old[b + j];
          int laps = j <= i ? L.laps_new[b + j] : L.laps_old[b + j];
          if (dis) continue;
          any = true;
          if (laps < 1) all = false;
        }
        if (any && all) pend = 1;
      }
    }
    P.env_i32[E_PENDING * P.E + env] = pend;
    pend_env = pend;
  }
  float o[22];
  float rew = 0.0f;
  if (env >= 0) {
    // _check_and_disable_cars (src/car_env.py:805-888)
    if (!c.disabled) {
      double speed = (double)vlen(c.v);
      if (speed < 0.5 && c.stuck_dur > 0) {
        double px = c.xf.p.x, py = c.xf.p.y;
        if (!c.has_stuck_start) { c.has_stuck_start = 1; c.stuck_sx = px; c.stuck_sy = py; }
        double dx = px - c.stuck_sx, dy = py - c.stuck_sy;
        double moved = PH(P2(dx) + P2(dy));
        if (c.stuck_dur > 10.0) {
          bool dis = false;
          if (moved < 1.0) dis = true;
          else if (c.stuck_dur > 15.0) dis = true;
          if (dis) { c.disabled = 1; c.just_disabled = 1; }
        }
      } else { c.stuck_dur = 0.0; c.has_stuck_start = 0; }
    }
    LPROF(3);
    car_obs(c, o);
    LPROF(4);
    // _calculate_multi_rewards (src/car_env.py:980-1113)
    if (c.disabled && !c.just_disabled) rew = 0.0f;
    else {
      double r = c.just_disabled ? 10.0 : 0.0;
      if (!c.disabled) r -= 0.05;
      if (!c.disabled) { double imp = c.imp_present ? c.imp : 0.0; if (fabs(imp) > 0) r -= 0.5; }
      double px = c.xf.p.x, py = c.xf.p.y;
      double dx = px - c.prev_px, dy = py - c.prev_py;
      r += PH(P2(dx) + P2(dy)) * 0.15;
      c.prev_px = px; c.prev_py = py;
      if (!c.first_step) {
        double prog = prog_now;
        double L = T.total_length, pd = prog - c.prog_hist;
        if (pd > L / 2) pd -= L; else if (pd < -L / 2) pd += L;
        if (pd < 0) {
          c.back += fabs(pd);
          if (c.back > 200.0 && !c.disabled) { c.disabled = 1; c.just_disabled = 1; }
          if (c.back > 25.0) {
            double ce = pymax(0.0, c.back - 25.0), pe = pymax(0.0, c.prev_back - 25.0);
            double nb = ce - pe;
            if (nb > 0) r -= nb * 0.05;
          }
        } else { c.back = 0.0; c.prev_back = 0.0; }
        c.prog_hist = prog;
      } else {
        c.prog_hist = prog_now;
        c.first_step = 0;
      }
      if (c.lt_laps > c.prev_laps) { r += 0.0 * (c.lt_laps - c.prev_laps); c.prev_laps = c.lt_laps; }
      if (!c.disabled) c.prev_back = c.back;
      rew = (float)r;
    }
    L.dis_final[tid] = c.disabled;
    L.below[tid] = (!c.disabled && c.cum_reward < -250.0f) ? 1 : 0;
  }
  LPROF(5);
  __syncthreads();
  // env pass 2: termination (src/car_env.py:1115-1158, 791-794)
  if (env >= 0 && car == 0) {
    const double st = sim + P.dt_d;   // env_time is written only here
    P.env_time[env] = st;
    int ndis = 0, active = 0, below = 0, term = 0, trunc = 0, reason = reason_in & 0xFF;
    for (int j0 = 0; j0 < C; j0 += 8) {   // 8 cars' words requested together per round
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (j0 + u >= C) break;
        const int d = L.dis_final[tid + j0 + u], b = L.below[tid + j0 + u];
        ndis += d;
        if (!d) { active++; below += b; }
      }
    }
    if (ndis >= C) { term = 1; reason = 1; }
    else if (active > 0 && below == active) { term = 1; reason = 2; }
    else if (P.reset_on_lap && st > 60.0) { term = 1; reason = 3; }
    else if (st > 180.0) { trunc = 1; reason = 4; }
    if (pend_env) { P.env_i32[E_PENDING * P.E + env] = 0; term = 1; }   // pass 1's value (same lane)
    P.env_i32[E_REASON * P.E + env] = reason;
    P.env_i32[E_TERMINATED * P.E + env] = term;
    P.env_i32[E_TRUNCATED * P.E + env] = trunc;
    int done = term | trunc;
    // bit 1: the env was never reset (E_CREATED == 0): an auto-reset builds it fresh worlds (read here, before
    // the barrier, because car 0 sets E_CREATED after its own reset below)
    L.envdone[el] = done | ((reason_in & 0x100) ? 2 : 0);
    if (env_flags) env_flags[env] = (uint8_t)((term ? EF_TERMINATED : 0) | (trunc ? EF_TRUNCATED : 0) |
                                              ((auto_reset && done) ? EF_RESET : 0) | ((reason & 7) << 4));
  }
  __syncthreads();
  if (env >= 0) {
    c.imp_at_obs = c.imp_present ? c.imp : 0.0;
    const bool collided = c.imp_at_obs != 0.0;
    c.cum_reward_info = c.cum_reward;
    c.imp = 0.0; c.imp_present = 1;                  // src/car_env.py:775-779
    c.cum_reward = c.cum_reward + rew;                // float32 accumulation (NEP 50)
    uint8_t flags = (uint8_t)((c.disabled ? CF_DISABLED : 0) | (c.just_disabled ? CF_JUST_DISABLED : 0) |
                              (collided ? CF_COLLISION : 0) | (lapdone ? CF_LAP : 0) | (c.overflow ? CF_ERROR : 0));
    c.just_disabled = 0;
    if (P.vhist) {   // Car.update_physics appends |v| at the start of the next step (src/car.py:384-386)
      const int k = (int)rint((sim + P.dt_d) * 60.0);
      P.vhist[(size_t)(k % VH_RING) * P.N + n] = vlen(c.v);
    }
    reward[n] = rew;
    if (car_flags) car_flags[n] = flags;
    const bool reset_now = auto_reset && (L.envdone[el] & 1);
    LPROF(6);
    if (terminal_obs) { float* t = terminal_obs + (size_t)n * 38; for (int i = 0; i < 22; ++i) t[i] = o[i]; }
    // sensor pass B: the reset pose of every auto-reset car (its pass-B values overwrite the pass-A ones in obs); the
    // env's reset byte tells the step's sensor passes which pass-B records are this step's
    if (car == 0) P.reset_env[env] = reset_now ? 1 : 0;
    if (reset_now) {
      // an env never reset before (E_CREATED == 0) gets fresh worlds, as in reset_kernel
      car_reset(P, c, n, (L.envdone[el] & 2) != 0, S, T);
      car_obs(c, o);
      set_pose(P, (size_t)P.N + n, c, PM_B_OBS);
    }
    // the lane's 88 bytes of obs[n, 0:22], stored directly (8-byte aligned rows: 11 float2 stores; staging the block's
    // rows in LDS for coalesced stores cost a barrier: per-shard model_logic_kernel 103.8 -> 102.5 us without it)
    for (int i = 0; i < 22; i += 2) *(float2*)(obs + (size_t)n * 38 + i) = make_float2(o[i], o[i + 1]);
    if (reset_now) car_store(P, n, c);    // car_reset rewrote every field
    else car_store_logic(P, n, c);
    LPROF(7);
    if (reset_now && car == 0) {
      P.env_time[env] = 0.0;
      P.env_i32[E_CREATED * P.E + env] = 1;
      P.env_i32[E_PENDING * P.E + env] = 0; P.env_i32[E_REASON * P.E + env] = 0;
      P.env_i32[E_TERMINATED * P.E + env] = 0; P.env_i32[E_TRUNCATED * P.E + env] = 0;
    }
  }
  LPROF(8);}

// ------------------------------------------------------------------ car-car contact (build-only extension)
// NOT in the reference: each reference car lives in its own b2World (src/car_physics.py:74-107) and its fixture's mask
// filters other cars out (src/constants/physics.py:9 COLLISION_MASK_CARS), so cars of one env never touch.
// With nascar_set_car_contact(h, 1) the cars of an env collide after their Box2D steps, with Box2D's contact algorithms
// for two dynamic bodies: every pair of car boxes whose centres are within two circumradii gets b2CollidePolygons'
// manifold (collide_polygons: 1-2 clip points, the same code as the wall contacts), and the env's touching pairs are
// solved by b2ContactSolver's sequential impulses -- per iteration and contact, the tangent (friction) impulses clamped
// by friction x normal impulse, then the normal impulses accumulated and clamped at >= 0, each applied to both cars'
// linear AND angular velocity (mass 1500 kg, the box's inertia) -- for BOX2D_VELOCITY_ITERATIONS (6), with the fixture
// mixing Box2D applies to a car pair: friction sqrt(0.7 * 0.7), restitution max(0.1, 0.1) (src/constants/car_specs.py:
// 39-40) as a velocity bias below -1 m/s relative normal speed (b2_velocityThreshold).  The accumulated normal impulses
// enter each car's collision impulse as CarCollisionListener.PostSolve does for walls (max over contact points), so
// damage and impact disables apply; a car that receives an impulse is woken.  What a shared b2World would do and this
// does not: the car-car constraints are solved after (not interleaved with) each car's wall island, with no warm start
// across steps, the 2-point block solver replaced by point-by-point sequential impulses, and no position correction (the
// per-car Box2D steps, their proxies and TOI sweeps are done; overlap is removed by the velocities over the next steps).
// One lane per env (its car 0) solves the env; the bodies and constraints sit in the caller's LDS scratch
// (CC_LDS_BYTES).  Sensors still see walls only.  Default off; every parity test runs with it off.
#define CAR_FRICTION_MIX 0.7f      // sqrt(CAR_FRICTION * CAR_FRICTION)
#define CAR_RESTITUTION_MIX 0.1f   // max(CAR_RESTITUTION, CAR_RESTITUTION)
#define CC_VELOCITY_ITERATIONS 6   // BOX2D_VELOCITY_ITERATIONS (src/constants/physics.py:16)
struct CCBody { V2 c; Rot q; V2 v; float w, jmax; };
struct CCon {                       // one touching car pair: b2ContactVelocityConstraint for two dynamic bodies
  int ia, ib, np; V2 n;
  V2 rA[2], rB[2]; float nm[2], tm[2], vb[2], ni[2], ti[2];
};
#define CC_LDS_BYTES ((size_t)SBLOCK * (sizeof(CCBody) + sizeof(CCon)))
#ifndef CC_FUSED
#define CC_FUSED 1   // the car-car phase inside model_logic_kernel (a call; 0: the two-launch path when it is on)
#endif
__device__ __attribute__((noinline)) void car_contact_env(CCBody* B, CCon* K, int C, int kcap) {
  Poly box; make_box(&box, CAR_HX, CAR_HY);
  int nk = 0;
  for (int i = 0; i < C; ++i)
    for (int j = i + 1; j < C; ++j) {
      const CCBody A = B[i], D = B[j];
      if (fabsf(D.c.x - A.c.x) > 5.7f || fabsf(D.c.y - A.c.y) > 5.7f) continue;   // > 2 circumradii apart
      Xf xa; xa.p = A.c; xa.q = A.q;
      Xf xb; xb.p = D.c; xb.q = D.q;
      DContact m;
      collide_polygons(m, &box, xa, &box, xb);
      if (m.pointCount == 0 || nk == kcap) continue;
      V2 nrm, pts[2];
      world_manifold(m, xa, xb, &nrm, pts);
      CCon k;
      k.ia = i; k.ib = j; k.np = m.pointCount; k.n = nrm;
      const V2 t = vcross_vs(nrm, 1.0f);
      for (int q = 0; q < 2; ++q) {
        k.ni[q] = 0.0f; k.ti[q] = 0.0f; k.nm[q] = 0.0f; k.tm[q] = 0.0f; k.vb[q] = 0.0f;
        k.rA[q] = zero2(); k.rB[q] = zero2();
        if (q >= k.np) continue;
        const V2 rA = vsub(pts[q], A.c), rB = vsub(pts[q], D.c);
        k.rA[q] = rA; k.rB[q] = rB;
        const float rnA = vcross(rA, nrm), rnB = vcross(rB, nrm);
        const float kn = CAR_INV_MASS + CAR_INV_MASS + CAR_INV_I * rnA * rnA + CAR_INV_I * rnB * rnB;
        k.nm[q] = kn > 0.0f ? fdiv_cr(1.0f, kn) : 0.0f;
        const float rtA = vcross(rA, t), rtB = vcross(rB, t);
        const float kt = CAR_INV_MASS + CAR_INV_MASS + CAR_INV_I * rtA * rtA + CAR_INV_I * rtB * rtB;
        k.tm[q] = kt > 0.0f ? fdiv_cr(1.0f, kt) : 0.0f;
        const V2 dv = vsub(vadd(D.v, vcross_sv(D.w, rB)), vadd(A.v, vcross_sv(A.w, rA)));
        const float vrel = vdot(nrm, dv);
        if (vrel < -VELOCITY_THRESHOLD) k.vb[q] = -CAR_RESTITUTION_MIX * vrel;
      }
      K[nk++] = k;
    }
  if (nk == 0) return;
  for (int it = 0; it < CC_VELOCITY_ITERATIONS; ++it)
    for (int kk = 0; kk < nk; ++kk) {
      CCon& k = K[kk];
      CCBody& A = B[k.ia];
      CCBody& D = B[k.ib];
      V2 vA = A.v, vB = D.v; float wA = A.w, wB = D.w;
      const V2 nrm = k.n, t = vcross_vs(nrm, 1.0f);
      for (int q = 0; q < k.np; ++q) {   // friction first, as b2ContactSolver::SolveVelocityConstraints
        const V2 dv = vsub(vadd(vB, vcross_sv(wB, k.rB[q])), vadd(vA, vcross_sv(wA, k.rA[q])));
        const float vt = vdot(dv, t);
        float lambda = k.tm[q] * (-vt);
        const float maxF = CAR_FRICTION_MIX * k.ni[q];
        const float ni = fclamp(k.ti[q] + lambda, -maxF, maxF);
        lambda = ni - k.ti[q];
        k.ti[q] = ni;
        const V2 Pt = vmul(lambda, t);
        vA = vsub(vA, vmul(CAR_INV_MASS, Pt)); wA -= CAR_INV_I * vcross(k.rA[q], Pt);
        vB = vadd(vB, vmul(CAR_INV_MASS, Pt)); wB += CAR_INV_I * vcross(k.rB[q], Pt);
      }
      for (int q = 0; q < k.np; ++q) {   // normal: accumulated impulse clamped at >= 0
        const V2 dv = vsub(vadd(vB, vcross_sv(wB, k.rB[q])), vadd(vA, vcross_sv(wA, k.rA[q])));
        const float vn = vdot(dv, nrm);
        float lambda = -k.nm[q] * (vn - k.vb[q]);
        const float ni = fmaxb(k.ni[q] + lambda, 0.0f);
        lambda = ni - k.ni[q];
        k.ni[q] = ni;
        const V2 Pn = vmul(lambda, nrm);
        vA = vsub(vA, vmul(CAR_INV_MASS, Pn)); wA -= CAR_INV_I * vcross(k.rA[q], Pn);
        vB = vadd(vB, vmul(CAR_INV_MASS, Pn)); wB += CAR_INV_I * vcross(k.rB[q], Pn);
      }
      A.v = vA; A.w = wA; D.v = vB; D.w = wB;
    }
  for (int kk = 0; kk < nk; ++kk) {   // CarCollisionListener.PostSolve: the largest normal impulse per car
    const CCon& k = K[kk];
    float j = 0.0f;
    for (int q = 0; q < k.np; ++q) j = fmaxb(j, k.ni[q]);
    B[k.ia].jmax = fmaxb(B[k.ia].jmax, j);
    B[k.ib].jmax = fmaxb(B[k.ib].jmax, j);
  }
}
// every thread of the block calls it (block barriers); scratch: CC_LDS_BYTES of LDS
__device__ __forceinline__ void car_contact_block(const Params& P, int tid, int el, int car, int env, int n,
                                                  unsigned char* scratch) {
  const int C = P.C;
  CCBody* B = (CCBody*)scratch;
  CCon* K = (CCon*)(scratch + (size_t)SBLOCK * sizeof(CCBody));
  if (env >= 0) {
    CCBody b;
    b.c = V(F32P(P, xpx)[n], F32P(P, xpy)[n]);      // (the body origin is its centre of mass)
    b.q.s = F32P(P, qs)[n]; b.q.c = F32P(P, qc)[n];
    b.v = V(F32P(P, vx)[n], F32P(P, vy)[n]); b.w = F32P(P, w)[n];
    b.jmax = 0.0f;
    B[tid] = b;
  }
  __syncthreads();
  if (env >= 0 && car == 0 && C > 1) car_contact_env(B + tid, K + tid, C, C);   // an env's C slots hold <= C contacts
  __syncthreads();
  if (env >= 0) {
    const CCBody b = B[tid];
    if (b.jmax > 0.0f) {
      F32P(P, vx)[n] = b.v.x; F32P(P, vy)[n] = b.v.y; F32P(P, w)[n] = b.w;
      if (!I32P(P, awake)[n]) { I32P(P, awake)[n] = 1; F32P(P, sleep)[n] = 0.0f; }
      if (!I32P(P, imp_present)[n]) { I32P(P, imp_present)[n] = 1; F64P(P, imp)[n] = 0.0; }
      F64P(P, imp)[n] = pymax(F64P(P, imp)[n], (double)b.jmax);
    }
  }
}
__global__ void __launch_bounds__(SBLOCK) car_contact_kernel(Params P) {
  const int tid = threadIdx.x, C = P.C;
  const int el = tid / C, car = tid - el * C;
  const int env = blk_env_of(P, el, wg_block(P) * P.epb + el);
  if (blk_empty(P, wg_block(P))) return;   // empty workgroup (device-built block map)
  car_contact_block(P, tid, el, car, env, env >= 0 ? env * C + car : 0, smem);
}

#ifndef LOGIC_WPE
#define LOGIC_WPE 0   // 0: the compiler's choice (182 VGPRs, 2 waves/SIMD)
#endif
#if LOGIC_WPE
#define LOGIC_ATTR __attribute__((amdgpu_waves_per_eu(LOGIC_WPE)))
#else
#define LOGIC_ATTR
#endif
__global__ void __launch_bounds__(SBLOCK) LOGIC_ATTR logic_kernel(Params P, float* obs, float* reward, uint8_t* car_flags,
                                                      uint8_t* env_flags, int auto_reset, float* terminal_obs) {
  __shared__ LogicLDS L;
  __shared__ TrackLDS TL;
  const int tid = threadIdx.x, C = P.C;
  const int el = tid / C, car = tid - el * C;
  const int slot = wg_block(P) * P.epb + el;
  const int env = blk_env_of(P, el, slot);
  const int n = env >= 0 ? env * C + car : 0;
  if (blk_empty(P, wg_block(P))) return;   // empty workgroup (device-built block map)
  PROF_B0(P.blk0);
  LPROF(0);
  Car c;
  double sim;
  int pend_in, reason_in;
  logic_load(P, env, car, n, c, sim, pend_in, reason_in);   // state loads issued before the staging barrier
  TrackDev T = P.tracks[blk_track_of(P, wg_block(P))];
  stage_track_lds(T, TL, tid);
  __syncthreads();
  T.segs = TL.segs; T.prefix = TL.prefix;
  logic_run(P, T, TL, L, tid, el, car, env, n, c, sim, pend_in, reason_in, obs, reward, car_flags, env_flags, auto_reset,
            terminal_obs);
}

// model_kernel + logic_kernel in one launch (NASCAR_FUSE_ML / nascar_set_fused_logic): each block runs its envs'
// logic as soon as ITS cars' Box2D steps are done (a block barrier) instead of after the whole grid's slowest
// wave, and one kernel boundary per step goes.  The logic's LDS (env reductions, obs rows, track segments) reuses
// the contact-slot region, free once every car of the block has written its contact records back.  Same device
// code as the two kernels, so the results are identical (tests run both).
struct FusedLogicLDS { LogicLDS L; TrackLDS TL; };
// the logic half of model_logic_kernel (inlined: out of line it spilled more, 39 vs 30 VGPRs)
#ifndef FUSED_LOGIC_NOINLINE
#define FUSED_LOGIC_NOINLINE 0
#endif
#if FUSED_LOGIC_NOINLINE
__attribute__((noinline))
#else
__forceinline__
#endif
static __device__ void fused_logic_phase(const Params& P, int tid, int el, int car, int env, int n, float* obs, float* reward,
                                         uint8_t* car_flags, uint8_t* env_flags, int auto_reset, float* terminal_obs,
                                         Car& c, double sim, int pend_in, int reason_in, const SegReg& sr) {
  FusedLogicLDS& F = *(FusedLogicLDS*)smem;
  if (env >= 0) logic_from_model(P, n, c);
  TrackDev T = P.tracks[blk_track_of(P, wg_block(P))];
  if (tid < T.nseg) { F.TL.prefix[tid] = sr.prefix; F.TL.sg[tid] = sr.sg; F.TL.rll[tid] = sr.rll; }   // (model half's loads)
  __syncthreads();
  PROF(7);
  T.segs = g_step_segs; T.prefix = F.TL.prefix;   // the segments the model half staged (static LDS, still there)
  logic_run(P, T, F.TL, F.L, tid, el, car, env, n, c, sim, pend_in, reason_in, obs, reward, car_flags, env_flags, auto_reset,
            terminal_obs);
}
#define MODEL_LOGIC_LDS_BYTES (MODEL_CT_LDS_BYTES > sizeof(FusedLogicLDS) ? MODEL_CT_LDS_BYTES : sizeof(FusedLogicLDS))
// one step of this workgroup's envs (model_logic_kernel; pipe_step_kernel runs it once per step of its loop)
__device__ __forceinline__ void model_logic_body(const Params& P, const void* actions, int discrete, int want_term, int policy,
                                                 uint64_t seed, int64_t step, const float* pobs, float* obs, float* reward,
                                                 uint8_t* car_flags, uint8_t* env_flags, int auto_reset, float* terminal_obs) {
  const int tid = threadIdx.x, C = P.C;
  const int el = tid / C, car = tid - el * C;
  const int slot = wg_block(P) * P.epb + el;
  const int env = blk_env_of(P, el, slot);
  const int n = env >= 0 ? env * C + car : 0;
  if (blk_empty(P, wg_block(P))) return;   // empty workgroup (device-built block map)
  Car c;
  SegReg sr;
  double sim;
  int pend_in, reason_in;
  logic_load_env(P, env, car, sim, pend_in, reason_in);
  model_block<true>(P, actions, discrete, want_term, policy, seed, step, pobs, tid, env, n, c, sr);
  __syncthreads();   // the block's Box2D steps done: body state stored, contact slots written back (LDS free)
  PROF(6);           // profile builds: the fused kernel's logic half (stamp slots 6-9)
#if CC_FUSED
  if (P.car_contact) car_contact_block(P, tid, el, car, env, n, smem);   // block-uniform; holds its own barriers
#endif
  fused_logic_phase(P, tid, el, car, env, n, obs, reward, car_flags, env_flags, auto_reset, terminal_obs, c, sim, pend_in,
                    reason_in, sr);
  PROF(8);
  PROF_RT(9);
}
__global__ void __launch_bounds__(SBLOCK) __attribute__((amdgpu_waves_per_eu(MODEL_WPE)))
model_logic_kernel(Params P, const void* actions, int discrete, int want_term, int policy, uint64_t seed, int64_t step,
                   const float* pobs, float* obs, float* reward, uint8_t* car_flags, uint8_t* env_flags, int auto_reset,
                   float* terminal_obs) {
  model_logic_body(P, actions, discrete, want_term, policy, seed, step, pobs, obs, reward, car_flags, env_flags, auto_reset,
                   terminal_obs);
}

// Fused multi-step rollout (nascar_rollout): K env steps of each block's envs in one launch, the actions
// from a device action source (policy 0 / 1 / 3, policy_car) on the previous step's observation.  Per step
// a block runs policy + model (one lane per car), logic (one lane per car, env passes in LDS) and the
// sensors (4 lanes per car in RAY_LPC rounds of the block's threads), with block barriers between the
// phases; the track's segments and sensor wall image are staged in LDS once per launch.  A car with a long
// Box2D chain (TOI events, contact islands) delays only its own block, which the other blocks do not wait
// for: in the per-step path every step waits for the slowest car of the whole batch.  Same device code as
// model_kernel / logic_kernel / ray_sensor_kernel, so the results equal K x (nascar_policy_actions +
// nascar_step with auto-reset) bit for bit (tests/test_gpu_rollout.py).
// Each phase is an out-of-line function: inlined into one loop, the three phases' loop-invariant addresses
// and live ranges spilled ~700 VGPRs; as calls each phase is allocated like its own kernel (the loop keeps
// only a few values live across them).  Params are read from a device copy (nascar_rollout uploads it)
// through a constant-address-space pointer, so the phases use scalar loads.  (The address of a by-value
// kernel argument must not be used for that: clang copies an address-taken argument to private memory.)
typedef const __attribute__((address_space(4))) Params* ParamsK;
__shared__ TrackLDS g_ro_track;    // rollout_kernel: the block's track segments
__shared__ LogicLDS g_ro_logic;    // rollout_kernel: logic_run's env reductions / obs rows

struct RoSlot { int tid, el, car, env, n; };
__device__ __forceinline__ RoSlot ro_slot(const Params& P) {
  RoSlot r;
  r.tid = threadIdx.x;
  r.el = r.tid / P.C; r.car = r.tid - r.el * P.C;
  r.env = blk_env_of(P, r.el, blockIdx.x * P.epb + r.el);
  r.n = r.env >= 0 ? r.env * P.C + r.car : 0;
  return r;
}
__device__ __forceinline__ TrackDev ro_track(const Params& P) {
  TrackDev T = P.tracks[blk_track_of(P, blockIdx.x)];
  T.segs = g_ro_track.segs; T.prefix = g_ro_track.prefix;
  return T;
}
static __device__ __attribute__((noinline)) void ro_model_phase(ParamsK Pk, int policy, uint64_t seed, int64_t step,
                                                                const float* obs) {
  const Params& P = *(const Params*)Pk;
  const RoSlot s = ro_slot(P);
  if (s.env < 0) return;
  const TrackDev T = ro_track(P);
  Car c;
  car_load_phys(P, s.n, c);
  c.pid = s.n;
  float tb, st;
  policy_car(policy, seed, step, s.n, obs, P.ctl, tb, st);
  model_car(P, c, s.n, T, tb, st, 0);
}
static __device__ __attribute__((noinline)) void ro_logic_phase(ParamsK Pk, float* obs, float* reward, uint8_t* car_flags,
                                                                uint8_t* env_flags, int auto_reset) {
  const Params& P = *(const Params*)Pk;
  const RoSlot s = ro_slot(P);
  const TrackDev T = ro_track(P);
  Car c;
  double sim;
  int pend_in, reason_in;
  logic_load(P, s.env, s.car, s.n, c, sim, pend_in, reason_in);
  logic_run(P, T, g_ro_track, g_ro_logic, s.tid, s.el, s.car, s.env, s.n, c, sim, pend_in, reason_in, obs, reward,
            car_flags, env_flags, auto_reset, nullptr);
}
static __device__ __attribute__((noinline)) void ro_contact_phase(ParamsK Pk) {
  const Params& P = *(const Params*)Pk;
  const RoSlot s = ro_slot(P);
  const TrackDev T = P.tracks[blk_track_of(P, blockIdx.x)];   // the scratch follows the staged sensor wall image
  car_contact_block(P, s.tid, s.el, s.car, s.env, s.n, smem + ((2 * (size_t)T.nwall * sizeof(float4) + 15) & ~(size_t)15));
}
static __device__ __attribute__((noinline)) void ro_sensor_phase(ParamsK Pk, float* obs, int passes) {
  const Params& P = *(const Params*)Pk;
  const TrackDev T = ro_track(P);
  ray_block_batched(P, T, (const float4*)smem, obs, passes);
}
__global__ void __launch_bounds__(SBLOCK) __attribute__((amdgpu_waves_per_eu(MODEL_WPE)))
rollout_kernel(const Params* __restrict__ Pg, int K, int policy, uint64_t seed, int64_t step0, float* obs, float* reward,
               uint8_t* car_flags, uint8_t* env_flags, int auto_reset, int traj) {
  ParamsK Pk = (ParamsK)Pg;   // global -> constant address space (same addresses)
  const Params& P = *Pg;
  if (blk_empty(P, blockIdx.x)) return;   // empty workgroup (device-built block map)
  PROF_B0(0);
  {
    const TrackDev T = P.tracks[blk_track_of(P, blockIdx.x)];
    stage_track_lds(T, g_ro_track, threadIdx.x);
    float4* s_w = (float4*)smem;   // [2 * nwall] sensor wall image
    for (int k = threadIdx.x; k < 2 * T.nwall; k += SBLOCK) s_w[k] = ldg(T.swall + k);
  }
  __syncthreads();
#pragma unroll 1
  for (int k = 0; k < K; ++k) {
    const size_t ko = traj ? (size_t)k : 0;
#ifdef NASCAR_PROFILE
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#endif
    ro_model_phase(Pk, policy, seed, step0 + k, obs);
    __syncthreads();
    if (P.car_contact) {
      ro_contact_phase(Pk);
      __syncthreads();
    }
#ifdef NASCAR_PROFILE
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
#endif
    ro_logic_phase(Pk, obs, reward + ko * P.N, car_flags ? car_flags + ko * P.N : nullptr,
                   env_flags ? env_flags + ko * P.E : nullptr, auto_reset);
    __syncthreads();
#ifdef NASCAR_PROFILE
    const unsigned long long t2 = __builtin_amdgcn_s_memtime();
#endif
    ro_sensor_phase(Pk, obs, auto_reset ? 3 : 1);
    __syncthreads();
#ifdef NASCAR_PROFILE
    const unsigned long long t3 = __builtin_amdgcn_s_memtime();
    RPROF_ADD(0, t1 - t0); RPROF_ADD(1, t2 - t1); RPROF_ADD(2, t3 - t2); RPROF_ADD(3, 1);
#endif
  }
}

// ------------------------------------------------------------------ pipelined rollout (nascar_set_rollout_pipe)
// K closed-loop steps with no per-step launch boundary: every step workgroup (pipe_step_kernel, one per env group, the
// rollout_kernel's model + logic phases) goes on to its next step as soon as its own sensors are done, and the sensors
// run in a second, high-occupancy persistent kernel (pipe_sensor_kernel, 52 VGPRs) that takes 8-car items from a device
// ring as the step workgroups publish them.  A slow car (a TOI chain) delays only its own group, not the step of the
// whole batch.  Hand-offs follow the agent-scope release / acquire form (MI355X_MICROARCH.md, inter-workgroup
// visibility): every storing wave drains its stores (vmcnt(0)), the workgroup barrier, one lane's release fence, then
// the flag; the consumer's one lane polls, acquires, and the workgroup barrier precedes every load.  The protocol does
// not depend on placement or residency: a sensor workgroup serves whatever item it claimed once it is published, and a
// step workgroup waits only on its own group's items; every wait is clock-bounded and flags the call failed
// (nascar_rollout_pipe_status) instead of hanging.  Same per-env code in the same order per env: results equal the
// per-step path bit for bit (tests/test_gpu_rollout.py).
struct PipeDev {
  // per XCD x: ring[x * cap .. ] of (seq << 32) | (workgroup << 5 | item) -- the sensor items published by the step
  // workgroups running on XCD x, served only by the sensor workgroups on XCD x, so every hand-off stays inside one
  // XCD's L2 (the per-XCD L2s are not coherent with each other)
  unsigned long long* ring;
  // ctr[x * 32 + 0] items claimed, [x * 32 + 1] slots reserved, [x * 32 + 2] items expected on XCD x (per call);
  // ctr[256] step workgroups registered (per call), ctr[288] sticky error flag
  unsigned* ctr;
  unsigned* sdone;            // [nblocks] sensor items completed per step workgroup (per call)
  unsigned seq, cap;          // this call's ring tag; slots per XCD (all of the call's items)
  int sub, nb;                // PIPE_CARS-car sensor items per step workgroup; step workgroups
  int dbg;                    // NASCAR_PIPE_DEBUG: printf milestones of the first workgroups
  unsigned long long timeout; // s_memrealtime ticks (100 MHz) a wait may last without progress (NASCAR_PIPE_TIMEOUT_MS)
};
#define PIPE_ERR 288
#define PIPE_REG 256
__device__ __forceinline__ unsigned pipe_ld(const unsigned* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void pipe_fail(const PipeDev& Q) { __hip_atomic_store(Q.ctr + PIPE_ERR, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
// agent-scope fences; NASCAR_PIPE_DEBUG bit 2 (value 4) makes them system-scope (diagnostic)
__device__ __forceinline__ void pipe_acquire(const PipeDev& Q) {
  if (Q.dbg & 4) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  else __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the invalidate completes asynchronously: wait for it
}
// producer side: the producer and the consumer share the XCD's L2 (per-XCD rings), and every storing wave has drained
// its stores into it (vmcnt(0)) before this, so the agent-scope release's L2 write-back (buffer_wbl2, which writes back
// the whole XCD L2's dirty lines, ~2-7 us) is not needed; NASCAR_PIPE_DEBUG bit 2 (4) keeps a system-scope release
__device__ __forceinline__ void pipe_release(const PipeDev& Q) {
  if (Q.dbg & 4) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
__device__ __forceinline__ unsigned pipe_xcc() { return __builtin_amdgcn_s_getreg((3 << 11) | 20) & 7u; }   // HW_REG_XCC_ID

// the step body as a call: allocated like model_logic_kernel on its own, not merged with the loop's live values
// (Params from the launch's device copy through a constant-address-space pointer, as rollout_kernel's phases: a
// by-value kernel argument whose address is taken would be copied to private memory)
static __device__ __attribute__((noinline)) void pipe_step_body(ParamsK Pk, int policy, uint64_t seed, int64_t step,
                                                                float* obs, float* reward, uint8_t* car_flags,
                                                                uint8_t* env_flags, int auto_reset) {
  const Params& P = *(const Params*)Pk;
  model_logic_body(P, nullptr, 0, 0, policy, seed, step, obs, obs, reward, car_flags, env_flags, auto_reset, nullptr);
}
__global__ void __launch_bounds__(SBLOCK) __attribute__((amdgpu_waves_per_eu(MODEL_WPE)))
pipe_step_kernel(const Params* __restrict__ Pg, PipeDev Q, int K, int policy, uint64_t seed, int64_t step0, float* obs,
                 float* reward, uint8_t* car_flags, uint8_t* env_flags, int auto_reset, int traj) {
  ParamsK Pk = (ParamsK)Pg;
  const Params& P = *Pg;
  const int b = wg_block(P), tid = threadIdx.x;
  const unsigned x = pipe_xcc();
  __shared__ int s_go;
  if (tid == 0) {   // this workgroup's items of the call go to its XCD's ring
    __hip_atomic_fetch_add(Q.ctr + x * 32 + 2, (unsigned)(Q.sub * K), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(Q.ctr + PIPE_REG, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (Q.dbg && b < 8) printf("pipe A b %d blockIdx %d xcc %u\n", b, (int)blockIdx.x, x);
  }
#pragma unroll 1
  for (int k = 0; k < K; ++k) {
    if (k > 0) {   // this group's sensors of step k - 1 done (the obs its driver reads, the state it steps)
      if (tid == 0) {
        const unsigned want = (unsigned)Q.sub * (unsigned)k;
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        int ok = 1;
        while (pipe_ld(Q.sdone + b) < want) {
          if (pipe_ld(Q.ctr + PIPE_ERR) || __builtin_amdgcn_s_memrealtime() - t0 > Q.timeout) { pipe_fail(Q); ok = 0; break; }
          __builtin_amdgcn_s_sleep(2);
        }
        pipe_acquire(Q);
        s_go = ok;
      }
      __syncthreads();
      if (Q.dbg && tid == 0 && b < 2) printf("pipe A b %d k %d go %d sdone %u\n", b, k, s_go, pipe_ld(Q.sdone + b));
      if (!__builtin_amdgcn_readfirstlane(s_go)) return;   // (wave-uniform, see pipe_sensor_kernel)
    }
    if (Q.dbg && tid == 0 && b < 2) printf("pipe A b %d k %d step\n", b, k);
    const size_t ko = traj ? (size_t)k : 0;
    pipe_step_body(Pk, policy, seed, step0 + k, obs, reward + ko * P.N, car_flags ? car_flags + ko * P.N : nullptr,
                   env_flags ? env_flags + ko * P.E : nullptr, auto_reset);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's stores done before the barrier and the release
    __syncthreads();
    if ((Q.dbg & 8) && tid == 0 && b < 2) {
      const int n0 = blk_env_of(P, 0, b * P.epb) * P.C;
      printf("pipe A b %d k %d car %d pose %f %f %f w %x\n", b, k, n0, P.pose[n0].x, P.pose[n0].y, P.pose[n0].z, __float_as_int(P.pose[n0].w));
      printf("pipe A b %d k %d car %d pose %f %f %f w %x\n", b, k, n0 + 33, P.pose[n0 + 33].x, P.pose[n0 + 33].y, P.pose[n0 + 33].z, __float_as_int(P.pose[n0 + 33].w));
    }
    if (tid == 0) {   // publish the group's sensor items of step k
      pipe_release(Q);
      const unsigned s0 = __hip_atomic_fetch_add(Q.ctr + x * 32 + 1, (unsigned)Q.sub, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      unsigned long long* R = Q.ring + (size_t)x * Q.cap;
      for (int j = 0; j < Q.sub; ++j)
        __hip_atomic_store(R + s0 + j, ((unsigned long long)Q.seq << 32) | (unsigned)(b << 5 | j), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      if (Q.dbg && b < 2) printf("pipe A b %d k %d published at %u\n", b, k, s0);
    }
  }
}

// 16 lanes per car, 4 cars per one-wave workgroup (so no workgroup barrier: the wave's own drained stores, then lane
// 0's release), walls read from the track's global image (ray_sensor_kernel's default path); loops over claimed items
// until the call's last.  The claimed item is read as a wave-uniform value (readfirstlane), so the loop's exit is a
// scalar branch.
#define PIPE_CARS 4
// one item's 4 cars, as a call: the loop around it keeps only a few values, and the walk's divergent control flow
// reconverges at the return (inlined into the item loop, lanes 1-15 of each car stayed off after the first item)
static __device__ __attribute__((noinline)) void pipe_sensor_item(ParamsK Pk, unsigned item, float* obs, int passes,
                                                                  int dbg) {
  const Params& P = *(const Params*)Pk;
  const int lane = threadIdx.x & 63, lc = lane / 16, r = lane % 16, C = P.C;
  const int b = (int)(item >> 5), slot = (int)(item & 31u) * PIPE_CARS + lc;
  if (slot < P.epb * C) {
    const int el = slot / C, car = slot - el * C;
    const int env = blk_env_of(P, el, b * P.epb + el);
    const TrackDev& T = P.tracks[blk_track_of(P, b)];
    if (env >= 0) {
      if (dbg & 2) ray_lane<16, true, false>(P, T, T.swall, env * C + car, r, obs, nullptr, passes);
      else ray_lane<16, true>(P, T, T.swall, env * C + car, r, obs, nullptr, passes);
    }
  }
}
// claiming an item and completing one as calls too: every lane enters and leaves each call with the whole wave
// active, and the item comes back wave-uniform.  (With the lane-0 regions inlined into the loop, the first item of a
// workgroup was walked right and later ones with only one lane of each car writing: the structurised loop did not
// restore the full exec mask before the next item's walk.)
static __device__ __attribute__((noinline)) unsigned pipe_claim(const PipeDev& Q, unsigned x) {
  unsigned item = 0xFFFFFFFFu;   // none left (or the call failed)
  if ((threadIdx.x & 63) == 0) {
    unsigned s = 0xFFFFFFFFu;
    unsigned* H = Q.ctr + x * 32;
    unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    // take the next slot of this XCD's ring (a queue in publication order); past the XCD's expected items (once every
    // step workgroup has registered them) there is nothing more to take
    const unsigned h = __hip_atomic_fetch_add(H, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (;;) {
      if (h < pipe_ld(H + 1)) { s = h; break; }   // reserved: its item is (being) published
      if (pipe_ld(Q.ctr + PIPE_REG) == (unsigned)Q.nb && h >= pipe_ld(H + 2)) break;
      if (pipe_ld(Q.ctr + PIPE_ERR) || __builtin_amdgcn_s_memrealtime() - t0 > Q.timeout) { pipe_fail(Q); break; }
      __builtin_amdgcn_s_sleep(4);
    }
    if (s != 0xFFFFFFFFu) {
      const unsigned long long* R = Q.ring + (size_t)x * Q.cap;
      t0 = __builtin_amdgcn_s_memrealtime();
      for (;;) {
        const unsigned long long v = __hip_atomic_load(R + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((unsigned)(v >> 32) == Q.seq) { item = (unsigned)v; break; }
        if (pipe_ld(Q.ctr + PIPE_ERR) || __builtin_amdgcn_s_memrealtime() - t0 > Q.timeout) { pipe_fail(Q); break; }
        __builtin_amdgcn_s_sleep(2);
      }
      pipe_acquire(Q);
    }
  }
  return __builtin_amdgcn_readfirstlane(item);
}
static __device__ __attribute__((noinline)) void pipe_done(const PipeDev& Q, int b) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the wave's obs stores done before the release
  if ((threadIdx.x & 63) == 0) {
    pipe_release(Q);
    __hip_atomic_fetch_add(Q.sdone + b, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(RSENSOR_WPE)))
pipe_sensor_kernel(const Params* __restrict__ Pg, PipeDev Q, float* obs, int passes) {
  ParamsK Pk = (ParamsK)Pg;
  const unsigned x = pipe_xcc();
#pragma unroll 1
  for (;;) {
    const unsigned item = pipe_claim(Q, x);
    if (item == 0xFFFFFFFFu) return;
    pipe_sensor_item(Pk, item, obs, passes, Q.dbg);
    if (Q.dbg & 16) pipe_sensor_item(Pk, item, obs, passes, Q.dbg);
    pipe_done(Q, (int)(item >> 5));
    if (Q.dbg & 32) return;
  }
}

__global__ void __launch_bounds__(SBLOCK) reset_kernel(Params P, const uint8_t* mask, float* obs) {
  const int tid = threadIdx.x, C = P.C;
  const int el = tid / C, car = tid - el * C;
  const int slot = blockIdx.x * P.epb + el;
  int env = blk_env_of(P, el, slot);
  if (blk_empty(P, blockIdx.x)) return;   // empty workgroup (device-built block map)
  if (env >= 0 && mask && !mask[env]) { P.pose[env * C + car] = make_float4(0.f, 0.f, 0.f, __int_as_float(0)); env = -1; }
  const TrackDev T = P.tracks[blk_track_of(P, blockIdx.x)];
  const WallSet S{T.walls, T.nwall, T.bp, T.sn, T.wfat};
  if (env >= 0) {
    const int n = env * C + car;
    const bool fresh = P.env_i32[E_CREATED * P.E + env] == 0;
    Car c;
    car_load(P, n, c);
    car_reset(P, c, n, fresh, S, T);
    float o[22];
    car_obs(c, o);
    for (int i = 0; i < 22; ++i) obs[(size_t)n * 38 + i] = o[i];
    set_pose(P, n, c, PM_A_OBS);
    car_store(P, n, c);
  }
  __syncthreads();   // every lane of an env has read E_CREATED before its car 0 writes it
  if (env >= 0 && car == 0) {
    P.env_time[env] = 0.0;
    P.env_i32[E_CREATED * P.E + env] = 1; P.env_i32[E_PENDING * P.E + env] = 0; P.env_i32[E_REASON * P.E + env] = 0;
    P.env_i32[E_TERMINATED * P.E + env] = 0; P.env_i32[E_TRUNCATED * P.E + env] = 0;
  }
}

__global__ void __launch_bounds__(SBLOCK) info_kernel(Params P, double* info) {
  const int tid = threadIdx.x, C = P.C;
  const int el = tid / C, car = tid - el * C;
  const int slot = blockIdx.x * P.epb + el;
  const int env = blk_env_of(P, el, slot);
  if (env < 0 || blk_track_of(P, blockIdx.x) < 0) return;
  const TrackDev T = P.tracks[blk_track_of(P, blockIdx.x)];
  const WallSet S{T.walls, T.nwall, T.bp, T.sn, T.wfat};
  const int n = env * C + car;
  Car c;
  car_load(P, n, c);
  double* o = info + (size_t)n * N_INFO;
  o[INFO_X] = c.xf.p.x; o[INFO_Y] = c.xf.p.y; o[INFO_VX] = c.v.x; o[INFO_VY] = c.v.y; o[INFO_ANGLE] = c.a; o[INFO_OMEGA] = c.w;
  o[INFO_SPEED] = (double)vlen(c.v); o[INFO_LAP_COUNT] = c.lt_laps;
  o[INFO_LAST_LAP] = c.lt_has_last ? c.lt_last : NAN; o[INFO_BEST_LAP] = c.lt_has_best ? c.lt_best : NAN;
  o[INFO_IS_TIMING] = c.lt_timing; o[INFO_CUR_LAP_TIME] = c.lt_cur; o[INFO_LAP_DIST] = c.lt_dist;
  o[INFO_HAS_CROSSED] = c.lt_crossed; o[INFO_DISABLED] = c.disabled; o[INFO_CUM_REWARD] = c.cum_reward_info;
  o[INFO_CUM_IMPACT] = c.cum_impact;
  o[INFO_ON_TRACK] = query_on_wall(S, c.xf.p.x, c.xf.p.y, 0.5) ? 0.0 : 1.0;
  o[INFO_RPM] = c.rpm; o[INFO_SIM_TIME] = P.env_time[env]; o[INFO_NCT] = c.nct; o[INFO_ERROR] = c.overflow;
  // CarEnv._calculate_track_progress of the current position (src/car_env.py:1544-1611): the reward pass
  // stores it every step for every car that is not disabled (and reset_car for the start pose)
  o[INFO_PROGRESS] = c.prog_hist;
  // Car.validate_performance inputs (src/car.py:1060-1098): the last min(k, 600) speeds (sample j = the speed
  // after j steps; sample 0, after the reset, is 0), their maximum and the position of the first one
  // >= CAR_TARGET_100KMH_MS in the window; the host turns them into the reference's dict (car_env.py)
  if (P.vhist) {
    const int k = (int)rint(P.env_time[env] * 60.0);
    const int cnt = k < VH_SIZE ? k : VH_SIZE, j0 = k - cnt;
    float mx = 0.0f; int first = -1;
    bool valid = true;
    for (int j = j0; j < k; ++j) {
      const float v = j == 0 ? 0.0f : P.vhist[(size_t)(j % VH_RING) * P.N + n];
      valid = valid && v == v;     // NaN: a slot not written since the history was enabled (mid-episode)
      if (j == j0 || v > mx) mx = v;
      if (first < 0 && (double)v >= 100.0 * 0.277778) first = j - j0;
    }
    if (valid) { o[INFO_PERF_COUNT] = cnt; o[INFO_PERF_MAX] = cnt ? (double)mx : 0.0; o[INFO_PERF_FIRST] = first; }
    else { o[INFO_PERF_COUNT] = -1.0; o[INFO_PERF_MAX] = 0.0; o[INFO_PERF_FIRST] = -1.0; }
  } else {
    o[INFO_PERF_COUNT] = -1.0; o[INFO_PERF_MAX] = 0.0; o[INFO_PERF_FIRST] = -1.0;
  }
}

// ------------------------------------------------------------------ random-track mode (CarEnv(track_file=None))
// CarEnv._select_random_track (src/car_env.py:264-287): a uniform choice over the bundled tracks, excluding the env's
// current track when it is one of them; every CarEnv.reset draws again (src/car_env.py:331-333) and a changed track
// gets fresh physics worlds (src/car_env.py:375-394).  learn/ppo.py:65-78 trains every env this way.  The reference
// re-seeds Python's global `random` from pid + wall clock before each draw, so its sequence is not reproducible; here
// draw k of an env is a counter hash of (the env's seed, k) -- reproducible on the host through nascar_track_draw.
__host__ __device__ inline uint32_t rt_mix32(uint64_t x) {   // splitmix64 finaliser
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  x ^= x >> 31;
  return (uint32_t)(x >> 32);
}
__host__ __device__ inline int rt_draw(uint64_t seed, int32_t k, int cur, const int* tracks, int nt) {
  if (nt <= 0) return cur;
  int pos = -1;
  for (int i = 0; i < nt; ++i) pos = (pos < 0 && tracks[i] == cur) ? i : pos;
  const bool excl = nt > 1 && pos >= 0;      // "if len(available_tracks) > 1 and previous_track in available_tracks"
  const uint32_t m = (uint32_t)(excl ? nt - 1 : nt);
  const uint32_t u = rt_mix32(seed ^ (0xD1B54A32D192ED03ull * ((uint64_t)(uint32_t)k + 1ull)));
  int j = (int)(((uint64_t)u * m) >> 32);    // uniform index into the candidates (random.choice)
  if (excl && j >= pos) ++j;
  return tracks[j];
}
// device state of the mode (nascar_set_random_tracks): per env its track, draws taken since seeding and seed
struct RtDev {
  int* env_track; int* draws; const uint64_t* seed; const int* tracks; int ntracks;
  int* dirty;   // set when an env changed track: block_map_kernel rebuilds the workgroup layout, then clears it
};
// nascar_reset: each reset env draws its next track; a changed one clears E_CREATED, so reset_kernel builds it fresh worlds
__global__ void __launch_bounds__(256) rt_reset_draw_kernel(Params P, RtDev R, const uint8_t* mask) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= P.E || (mask && !mask[e])) return;
  const int cur = R.env_track[e], k = R.draws[e];
  R.draws[e] = k + 1;
  const int t = rt_draw(R.seed[e], k, cur, R.tracks, R.ntracks);
  if (t != cur) {
    R.env_track[e] = t;
    P.env_i32[E_CREATED * P.E + e] = 0;
    *R.dirty = 1;
  }
}
// After a step with auto-reset: every env the step reset (env flag EF_RESET: reset in the launch on its old track) draws
// its next track; an env whose track changes is reset again on the new one with fresh worlds (Car() + CarPhysics,
// exactly reset_kernel's fresh path: every car field rewritten), its reset observation rewritten (obs[0:22] here, the 16
// sensors by pass-B ray walks on the new track).  A 256-thread workgroup per 64 envs: the first wave draws (one lane per
// env) and lists the switching envs in LDS; then every thread takes one car of them for the reset and one ray of them
// for the walks, so an env's whole reset and sensor work run in parallel (few envs switch per step: one per episode).
// The terminal observation (the old track's, written by the step) is untouched.
#define RT_SWITCH_BLOCK 256
__global__ void __launch_bounds__(RT_SWITCH_BLOCK) rt_switch_kernel(Params P, RtDev R, const uint8_t* env_flags, float* obs) {
  __shared__ int s_env[64], s_tr[64], s_n;
  const int tid = threadIdx.x, C = P.C;
  if (tid < 64) {
    const int e = blockIdx.x * 64 + tid;
    int nt = -1;
    if (e < P.E && (env_flags[e] & EF_RESET)) {
      const int cur = R.env_track[e], k = R.draws[e];
      R.draws[e] = k + 1;
      const int t = rt_draw(R.seed[e], k, cur, R.tracks, R.ntracks);
      if (t != cur) { R.env_track[e] = t; nt = t; }
    }
    const unsigned long long m = __ballot(nt >= 0);
    const int lane = tid;
    if (nt >= 0) {
      const int q = __popcll(m & (lane ? (~0ull >> (64 - lane)) : 0ull));
      s_env[q] = e; s_tr[q] = nt;
    }
    if (lane == 0) { s_n = __popcll(m); if (m) *R.dirty = 1; }
  }
  __syncthreads();
  const int ns = s_n;
  if (ns == 0) return;                    // (block-uniform)
  for (int t = tid; t < ns * C; t += RT_SWITCH_BLOCK) {   // one car per thread: the fresh reset on the new track
    const int q = t / C, car = t - q * C, n = s_env[q] * C + car;
    const TrackDev T = P.tracks[s_tr[q]];   // segments from global memory (as reset_kernel)
    const WallSet S{T.walls, T.nwall, T.bp, T.sn, T.wfat};
    Car c;
    car_load(P, n, c);
    car_reset(P, c, n, true, S, T);
    float o[22];
    car_obs(c, o);
    for (int i = 0; i < 22; ++i) obs[(size_t)n * 38 + i] = o[i];
    set_pose(P, (size_t)P.N + n, c, PM_B_OBS);
    car_store(P, n, c);
  }
  __threadfence();
  __syncthreads();                        // the pass-B poses stored before the walks read them
  for (int t0 = 0; t0 < ns * C * 16; t0 += RT_SWITCH_BLOCK) {   // one ray per thread (block-uniform loop), each
    const int t = t0 + tid;                                     // walking its whole list on its own lane
    if (t < ns * C * 16) {
      const int cc = t >> 4, q = cc / C, car = cc - q * C;
      const TrackDev T = P.tracks[s_tr[q]];
      ray_lane<16, true, false>(P, T, T.swall, s_env[q] * C + car, t & 15, obs, nullptr, 2);
    }
  }
}
// The workgroup layout rebuilt on the device (random-track mode; prepare() builds it on the host otherwise): envs
// grouped by track in ascending env order, each track's envs in whole workgroups of epb envs, tracks in id order, the
// workgroups past the last one empty (track -1) -- the host layout's order, with a fixed grid of nb_cap workgroups so
// no launch waits for the host.  One 1024-thread workgroup: per-track counts (LDS atomics), block offsets, then each
// env's rank among its track's envs by ballots over 1024-env chunks.  Does nothing unless *dirty (or force).
#define RT_MAX_TRACKS 64
// word w of a thread's packed per-track counts: tracks 2w (low 16 bits) and 2w + 1 (high 16 bits)
__device__ __forceinline__ uint32_t pk_get(const uint32_t c[4], int t) {
  const uint32_t w = (t >> 1) == 0 ? c[0] : (t >> 1) == 1 ? c[1] : (t >> 1) == 2 ? c[2] : c[3];
  return (t & 1) ? w >> 16 : w & 0xFFFFu;
}
__device__ __forceinline__ void pk_add(uint32_t c[4], int t, uint32_t v) {
  const uint32_t inc = v << ((t & 1) * 16);
#pragma unroll
  for (int w = 0; w < 4; ++w) c[w] += (t >> 1) == w ? inc : 0u;
}
__global__ void __launch_bounds__(1024) block_map_kernel(int E, int epb, int ntr, const int* env_track, int* blk_track,
                                                         int* blk_env, int nb_cap, int* dirty, int force) {
  __shared__ int cnt[RT_MAX_TRACKS], boff[RT_MAX_TRACKS + 1], run[RT_MAX_TRACKS], woff[16][RT_MAX_TRACKS];
  __shared__ uint32_t s_wt[16][4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (!force && *dirty == 0) return;      // (every thread reads it before thread 0 clears it, after the barriers below)
  auto track_of = [&](int b) {
    int tr = -1;
    for (int t = 0; t < ntr; ++t) tr = (b >= boff[t] && b < boff[t + 1]) ? t : tr;
    return tr;
  };
  if (ntr <= 8 && E < 65536) {
    // Fast path (up to 8 tracks: the bundled ones): thread t owns envs [t R, t R + R); its per-track counts packed as
    // 16-bit fields in 4 words, one block-wide exclusive scan of the packed words (wave scan by shuffles, then the 16
    // wave totals from LDS), so every env's slot comes out of one pass with a single barrier.
    const int R = (E + 1023) / 1024, e0 = tid * R;
    uint32_t c[4] = {0u, 0u, 0u, 0u};
    for (int i = 0; i < R; ++i) {
      const int e = e0 + i;
      if (e < E) pk_add(c, env_track[e], 1u);
    }
    uint32_t incl[4] = {c[0], c[1], c[2], c[3]};
#pragma unroll
    for (int d = 1; d < 64; d <<= 1)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t x = (uint32_t)__shfl_up((int)incl[k], d);
        if (lane >= d) incl[k] += x;
      }
    if (lane == 63) { s_wt[w][0] = incl[0]; s_wt[w][1] = incl[1]; s_wt[w][2] = incl[2]; s_wt[w][3] = incl[3]; }
    __syncthreads();
    uint32_t before[4] = {0u, 0u, 0u, 0u}, total[4] = {0u, 0u, 0u, 0u};
    for (int ww = 0; ww < 16; ++ww)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t x = s_wt[ww][k];
        before[k] += ww < w ? x : 0u;
        total[k] += x;
      }
    uint32_t ex[4];   // this thread's first rank within each track
#pragma unroll
    for (int k = 0; k < 4; ++k) ex[k] = before[k] + incl[k] - c[k];
    int bo[9];        // block offsets of the tracks (every thread computes them)
    bo[0] = 0;
#pragma unroll
    for (int t = 0; t < 8; ++t) bo[t + 1] = bo[t] + (t < ntr ? (int)((pk_get(total, t) + epb - 1) / epb) : 0);
    if (tid <= 8) boff[tid] = bo[tid];
    for (int i = 0; i < R; ++i) {
      const int e = e0 + i;
      if (e >= E) break;
      const int t = env_track[e];
      int b0 = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) b0 = t == k ? bo[k] : b0;
      blk_env[b0 * epb + (int)pk_get(ex, t)] = e;
      pk_add(ex, t, 1u);
    }
    __syncthreads();   // boff published
    for (int b = tid; b < nb_cap; b += 1024) blk_track[b] = track_of(b);
    for (int s = tid; s < ntr * epb; s += 1024) {   // the unfilled tail of each track's last workgroup
      const int t = s / epb, k = s - t * epb;
      const int n = (int)pk_get(total, t), tail = (boff[t + 1] - boff[t]) * epb - n;
      if (k < tail) blk_env[boff[t] * epb + n + k] = -1;
    }
    if (tid == 0) *dirty = 0;
    return;
  }
  for (int t = tid; t < ntr; t += 1024) { cnt[t] = 0; run[t] = 0; }
  __syncthreads();
  for (int e = tid; e < E; e += 1024) atomicAdd(&cnt[env_track[e]], 1);
  __syncthreads();
  if (tid == 0) {
    int b = 0;
    for (int t = 0; t < ntr; ++t) { boff[t] = b; b += (cnt[t] + epb - 1) / epb; }
    boff[ntr] = b;
  }
  __syncthreads();
  for (int b = tid; b < nb_cap; b += 1024) blk_track[b] = track_of(b);
  // the unfilled tail of each track's last workgroup (workgroups of track -1 are never read: every kernel returns first)
  for (int s = tid; s < ntr * epb; s += 1024) {
    const int t = s / epb, k = s - t * epb, tail = (boff[t + 1] - boff[t]) * epb - cnt[t];
    if (k < tail) blk_env[boff[t] * epb + cnt[t] + k] = -1;
  }
  const unsigned long long below = lane ? (~0ull >> (64 - lane)) : 0ull;
  for (int c0 = 0; c0 < E; c0 += 1024) {
    const int e = c0 + tid;
    const int t = e < E ? env_track[e] : -1;
    int rk = 0;
    for (int tt = 0; tt < ntr; ++tt) {
      const unsigned long long mm = __ballot(t == tt);
      if (lane == 0) woff[w][tt] = __popcll(mm);
      if (t == tt) rk = __popcll(mm & below);
    }
    __syncthreads();
    if (tid < ntr) {   // exclusive scan over the 16 waves, continuing the previous chunks' count
      int r = run[tid];
      for (int ww = 0; ww < 16; ++ww) { const int x = woff[ww][tid]; woff[ww][tid] = r; r += x; }
      run[tid] = r;
    }
    __syncthreads();
    if (t >= 0) blk_env[boff[t] * epb + woff[w][t] + rk] = e;
    __syncthreads();
  }
  if (tid == 0) *dirty = 0;
}

// ------------------------------------------------------------------ SB3 VecEnv bookkeeping (VecCarEnv, device tensors)
// The per-step work of SB3's Monitor + VecEnv around CarEnv.step (stable_baselines3 Monitor.step: the episode return as
// the float64 sum of the float32 rewards, the episode length; learn/ppo.py:65-78 wraps every env in Monitor) in one
// launch: done = terminated | truncated; the running return / length advanced, their values at this step written to
// the caller's snapshot buffers (what info["episode"] reports for an env that finished), then zeroed for finished envs.
__global__ void __launch_bounds__(256) vec_post_kernel(int E, int C, const float* reward, const uint8_t* env_flags,
                                                       double* ep_ret, int64_t* ep_len, uint8_t* done, double* snap_ret,
                                                       int64_t* snap_len) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  const bool d = (env_flags[e] & (EF_TERMINATED | EF_TRUNCATED)) != 0;
  for (int c = 0; c < C; ++c) {
    const size_t n = (size_t)e * C + c;
    const double r = ep_ret[n] + (double)reward[n];
    snap_ret[n] = r;
    ep_ret[n] = d ? 0.0 : r;
  }
  const int64_t l = ep_len[e] + 1;
  snap_len[e] = l;
  ep_len[e] = d ? 0 : l;
  done[e] = d ? 1 : 0;
}
// BaseEnv action-space check (assert self.action_space.contains(action), src/car_env.py:694): any action outside
// [-1, 1] (or NaN), or a discrete one outside {0..4}, sets *bad (read by the caller whenever it synchronises).
__global__ void __launch_bounds__(256) action_check_kernel(int n, const void* actions, int discrete, int* bad) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  bool b;
  if (discrete) { const int a = ((const int*)actions)[i]; b = a < 0 || a > 4; }
  else { const float a = ((const float*)actions)[i]; b = !(a >= -1.0f && a <= 1.0f); }
  if (b) *bad = 1;
}

// ------------------------------------------------------------------ synthetic action sources (bench)
// =================================================================== host side / C ABI
static thread_local std::string g_err;
static int fail(const char* fmt, ...) {
  char buf[512];
  va_list ap; va_start(ap, fmt); vsnprintf(buf, sizeof buf, fmt, ap); va_end(ap);
  g_err = buf;
  return -1;
}
#define HIPCHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) return fail("%s failed: %s", #x, hipGetErrorString(e_)); } while (0)

// persistent actor grid: one workgroup per CU (W2 fills the LDS), never more than the tiles
static int actor_grid(int n) {
  static int cus = 0;
  if (!cus) { int dev = 0; hipGetDevice(&dev); hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev); if (cus <= 0) cus = 256; }
  const int tiles = (n + 32 * ACT_WAVES - 1) / (32 * ACT_WAVES);   // >= one tile per wave
  return std::max(1, std::min(tiles, cus));
}


struct HostGrid {
  WallGrid g{};
  std::vector<int> start; std::vector<uint16_t> idx;
  int* d_start = nullptr; uint16_t* d_idx = nullptr;
  std::vector<float4> box; float4* d_box = nullptr;
};
// host-side wall record: the device's LWall plus the values only the host builders use
struct HWall : LWall {
  float rad;                 // bounding radius + culling margin (sensor wall image)
  float flx, fly, fhx, fhy;  // broadphase fat AABB
};
struct HostTrack {
  std::vector<HWall> walls; std::vector<DSeg> segs; std::vector<double> prefix;
  double total_length; int startline, has_banking;
  LWall* d_walls = nullptr; float4* d_wfat = nullptr; DSeg* d_segs = nullptr; double* d_prefix = nullptr;
  HostGrid bp, sn;
  struct {
    BeamGrid g{};
    std::vector<int4> chunk; std::vector<uint16_t> ent; std::vector<uint2> head;
    int4* d_chunk = nullptr; uint16_t* d_ent = nullptr; uint2* d_head = nullptr;
    int nxc = 0;
    size_t entries = 0, nlist = 0, dropped = 0;   // dropped: cells whose continuations overflow the 16-bit offsets
    double build_s = 0.0;
  } beam;
  std::vector<float4> groups; float4* d_groups = nullptr;
  float4* d_swall = nullptr;
};

// Wall grids (see WallGrid in nascar_device.h).  Conservative by construction: the
// broadphase list of a cell holds every wall whose fat AABB overlaps the cell grown by
// reach (+5 cm); the sensor list every wall whose culling circle (rad + 0.25 m) comes
// within 251 m of the cell, nearest first.
static const float BP_CELL = 4.0f, BP_REACH = 7.0f, SN_CELL = 16.0f, SN_PAD = 20.0f;
static const double SN_GROUP_R = 12.0; static const int SN_GROUP_N = 8;
static void build_grids(HostTrack& t) {
  double lx = 1e30, ly = 1e30, hx = -1e30, hy = -1e30;
  for (auto& w : t.walls) { lx = std::min(lx, (double)w.flx); ly = std::min(ly, (double)w.fly);
                            hx = std::max(hx, (double)w.fhx); hy = std::max(hy, (double)w.fhy); }
  auto setup = [&](HostGrid& G, float cell, float pad, float reach) {
    G.g.ox = (float)(lx - pad); G.g.oy = (float)(ly - pad); G.g.inv_cell = 1.0f / cell; G.g.reach = reach;
    G.g.nx = (int)std::ceil((hx + pad - G.g.ox) / cell) + 1; G.g.ny = (int)std::ceil((hy + pad - G.g.oy) / cell) + 1;
    G.start.assign((size_t)G.g.nx * G.g.ny + 1, 0);
  };
  setup(t.bp, BP_CELL, BP_REACH + 4.0f, BP_REACH);
  setup(t.sn, SN_CELL, SN_PAD, 0.0f);
  const int nw = (int)t.walls.size();
  for (int cy = 0; cy < t.bp.g.ny; ++cy)
    for (int cx = 0; cx < t.bp.g.nx; ++cx) {
      const double x0 = t.bp.g.ox + (double)cx * BP_CELL - BP_REACH - 0.05, x1 = t.bp.g.ox + (double)(cx + 1) * BP_CELL + BP_REACH + 0.05;
      const double y0 = t.bp.g.oy + (double)cy * BP_CELL - BP_REACH - 0.05, y1 = t.bp.g.oy + (double)(cy + 1) * BP_CELL + BP_REACH + 0.05;
      t.bp.start[(size_t)cy * t.bp.g.nx + cx] = (int)t.bp.idx.size();
      for (int j = 0; j < nw; ++j) {
        const HWall& w = t.walls[j];
        if (w.flx > x1 || w.fhx < x0 || w.fly > y1 || w.fhy < y0) continue;
        t.bp.idx.push_back((uint16_t)j);
        t.bp.box.push_back(make_float4(w.flx, w.fly, w.fhx, w.fhy));
      }
    }
  t.bp.start.back() = (int)t.bp.idx.size();
  for (int k = 0; k < std::max(BP_BATCH, 1); ++k) t.bp.box.push_back(make_float4(1e30f, 1e30f, -1e30f, -1e30f));
  // sensor wall groups: runs of consecutive walls (index order follows each boundary through
  // the curves) whose corners fit in a circle of radius <= SN_GROUP_R, at most SN_GROUP_N walls
  {
    auto corners = [&](int j, double* xs, double* ys) {
      const LWall& w = t.walls[j];
      const float vx[4] = {-w.hx, w.hx, w.hx, -w.hx}, vy[4] = {-w.hy, -w.hy, w.hy, w.hy};
      for (int i = 0; i < 4; ++i) { xs[i] = (w.qc * vx[i] - w.qs * vy[i]) + w.px; ys[i] = (w.qs * vx[i] + w.qc * vy[i]) + w.py; }
    };
    auto circle = [&](int first, int count, double& cx, double& cy) {
      double lx = 1e30, ly = 1e30, ux = -1e30, uy = -1e30, xs[4], ys[4];
      for (int j = first; j < first + count; ++j) {
        corners(j, xs, ys);
        for (int i = 0; i < 4; ++i) { lx = std::min(lx, xs[i]); ux = std::max(ux, xs[i]); ly = std::min(ly, ys[i]); uy = std::max(uy, ys[i]); }
      }
      cx = 0.5 * (lx + ux); cy = 0.5 * (ly + uy);
      double r = 0.0;
      for (int j = first; j < first + count; ++j) {
        corners(j, xs, ys);
        for (int i = 0; i < 4; ++i) r = std::max(r, std::hypot(xs[i] - cx, ys[i] - cy));
      }
      return r;
    };
    t.groups.clear();
    int first = 0;
    while (first < nw) {
      int count = 1;
      while (first + count < nw && count < SN_GROUP_N) {
        double cx, cy;
        if (circle(first, count + 1, cx, cy) > SN_GROUP_R) break;
        ++count;
      }
      double cx, cy, r = circle(first, count, cx, cy);
      const int packed = first | (count << 16);
      float pf; memcpy(&pf, &packed, sizeof pf);
      t.groups.push_back(make_float4((float)cx, (float)cy, (float)(r + 0.3), pf));
      first += count;
    }
  }
  std::vector<std::pair<double, int>> cand;
  const int ng = (int)t.groups.size();
  for (int cy = 0; cy < t.sn.g.ny; ++cy)
    for (int cx = 0; cx < t.sn.g.nx; ++cx) {
      const double x0 = t.sn.g.ox + (double)cx * SN_CELL, x1 = x0 + SN_CELL;
      const double y0 = t.sn.g.oy + (double)cy * SN_CELL, y1 = y0 + SN_CELL;
      const double mx = 0.5 * (x0 + x1), my = 0.5 * (y0 + y1);
      t.sn.start[(size_t)cy * t.sn.g.nx + cx] = (int)t.sn.idx.size();
      cand.clear();
      for (int g = 0; g < ng; ++g) {
        const float4 G = t.groups[g];
        const double dx = std::max(std::max(x0 - G.x, 0.0), G.x - x1), dy = std::max(std::max(y0 - G.y, 0.0), G.y - y1);
        if (std::sqrt(dx * dx + dy * dy) > 251.0 + G.z) continue;
        cand.push_back({std::hypot(G.x - mx, G.y - my) - G.z, g});
      }
      std::sort(cand.begin(), cand.end());
      for (auto& c : cand) t.sn.idx.push_back((uint16_t)c.second);
    }
  t.sn.start.back() = (int)t.sn.idx.size();
}
// Beam lists (BeamGrid).  Cells of `cell` m (BEAM_CELL_M by default) over the walls' extent; a cell gets lists when its centre is
// within (largest half width + BEAM_BAND) of a wall centre line -- the corridor and a band outside each wall.
// Per cell (centre c, disk radius rc = half diagonal + 5 cm) and wall j (centre line AB, capsule radius
// rr = half thickness + 10 cm, which holds the box and the f32 rounding of the device's ray cast):
//  * lb = dist(c, AB) - rr - rc bounds the distance from any ray origin in the cell to any point of the box;
//    walls with lb > 251 m are out of the 250 m ray's reach;
//  * the directions from the disk to the capsule lie in the arc between the directions from c to A and to
//    B, widened by asin((rr + rc) / dist(c, AB)) (all bins when c is inside the grown capsule), plus a
//    2e-3 rad guard for the f32 ray end points; every bin that arc touches lists the wall.
// Both are conservative, so the walk in ray_sensor_kernel visits every wall that can be the first hit.
// Cell size: the cell's disk widens every wall's angular arc and lowers its distance bound, so smaller cells give
// shorter walks (steady-state sensor tails; bench step 191 -> 178 / 174 / 168 / 167 us at 2 / 1.5 / 1 / 0.75 m,
// tools/ab2.sh) at 0.2-0.5 GB of lists per track at 1 m (8-byte heads + sentinel-terminated continuations).
#ifndef BEAM_CELL_M
#define BEAM_CELL_M 1.0f
#endif
#define BEAM_CELL_MIN 0.5f    // nascar_set_beam_cell range (heads: cell count x 4 KB; walks: longer above ~2 m)
#define BEAM_CELL_MAX 8.0f
static const double BEAM_BAND = 8.0;
static void build_beams(HostTrack& t, const float cell) {
  auto t0 = std::chrono::steady_clock::now();
  auto& B = t.beam;
  const int nw = (int)t.walls.size();
  std::vector<double> ax(nw), ay(nw), bx(nw), by(nw), rr(nw);
  double lx = 1e30, ly = 1e30, ux = -1e30, uy = -1e30, hwmax = 0.0;
  for (int j = 0; j < nw; ++j) {
    const LWall& w = t.walls[j];
    const double ex = (double)w.hx * w.qc, ey = (double)w.hx * w.qs;
    ax[j] = w.px - ex; ay[j] = w.py - ey; bx[j] = w.px + ex; by[j] = w.py + ey;
    rr[j] = (double)w.hy + 0.1;
    lx = std::min({lx, ax[j], bx[j]}); ux = std::max({ux, ax[j], bx[j]});
    ly = std::min({ly, ay[j], by[j]}); uy = std::max({uy, ay[j], by[j]});
  }
  for (auto& s : t.segs) hwmax = std::max(hwmax, s.width / 2.0);
  const double D = hwmax + BEAM_BAND, pad = D + 2.0 * cell;
  B.g.ox = (float)(lx - pad); B.g.oy = (float)(ly - pad); B.g.inv_cell = 1.0f / cell;
  B.g.nx = (int)std::ceil((ux + pad - B.g.ox) / cell) + 1;
  B.g.ny = (int)std::ceil((uy + pad - B.g.oy) / cell) + 1;
  const int nx = B.g.nx, ny = B.g.ny;
  auto segdist = [&](int j, double x, double y) {
    const double sx = bx[j] - ax[j], sy = by[j] - ay[j], ll = sx * sx + sy * sy;
    double tt = ll > 0 ? ((x - ax[j]) * sx + (y - ay[j]) * sy) / ll : 0.0;
    tt = std::min(1.0, std::max(0.0, tt));
    return std::hypot(x - (ax[j] + tt * sx), y - (ay[j] + tt * sy));
  };
  auto centre = [&](int cx, int cy, double& x, double& y) {
    x = (double)B.g.ox + (cx + 0.5) * (double)cell; y = (double)B.g.oy + (cy + 0.5) * (double)cell;
  };
  // cells near a wall
  std::vector<uint8_t> mark((size_t)nx * ny, 0);
  for (int j = 0; j < nw; ++j) {
    const int x0 = std::max(0, (int)std::floor((std::min(ax[j], bx[j]) - D - B.g.ox) / cell) - 1);
    const int x1 = std::min(nx - 1, (int)std::floor((std::max(ax[j], bx[j]) + D - B.g.ox) / cell) + 1);
    const int y0 = std::max(0, (int)std::floor((std::min(ay[j], by[j]) - D - B.g.oy) / cell) - 1);
    const int y1 = std::min(ny - 1, (int)std::floor((std::max(ay[j], by[j]) + D - B.g.oy) / cell) + 1);
    for (int cy = y0; cy <= y1; ++cy)
      for (int cx = x0; cx <= x1; ++cx) {
        double x, y;
        centre(cx, cy, x, y);
        if (segdist(j, x, y) <= D) mark[(size_t)cy * nx + cx] = 1;
      }
  }
  // entry layout: 10 wall bits up to 1024 walls (6-bit codes of c^2 / 16 m), then one more per doubling; the code scale
  // keeps the largest non-sentinel code near 240 m (a 250 m ray)
  uint32_t wb = 10;
  while (wb < BEAM_MAX_WALL_BITS && nw > (1 << wb)) ++wb;
  B.g.wbits = wb; B.g.wmask = (1u << wb) - 1u; B.g.cmax = (1u << (16 - wb)) - 1u;
  B.g.kq = (float)(0.0625 * std::pow(62.0 / (double)(B.g.cmax - 1), 2.0));
  std::vector<int> cells;   // the marked cells, row-major
  if (nw <= (1 << BEAM_MAX_WALL_BITS))   // (more walls than the entries address: no lists, the wall-group walk)
    for (size_t k = 0; k < mark.size(); ++k)
      if (mark[k]) cells.push_back((int)k);
  const int ncell = (int)cells.size();
  const double rc = cell * 0.70710678 + 0.05, two_pi = 2.0 * M_PI, dbin = two_pi / BEAM_NB;
  std::vector<std::vector<uint32_t>> lists((size_t)ncell * BEAM_NB);
  auto work = [&](int c0, int c1) {
    for (int ci = c0; ci < c1; ++ci) {
      double x, y;
      centre(cells[ci] % nx, cells[ci] / nx, x, y);
      std::vector<uint32_t>* L = &lists[(size_t)ci * BEAM_NB];
      for (int j = 0; j < nw; ++j) {
        const double d = segdist(j, x, y), R = rr[j] + rc, lb = d - R;
        if (lb > 251.0) continue;
        const uint32_t q = (uint32_t)std::min(65535.0, std::floor(std::max(lb, 0.0) * 100.0));
        const uint32_t e = (q << 16) | (uint32_t)j;
        if (d <= R * 1.0001 + 1e-3) { for (int k = 0; k < BEAM_NB; ++k) L[k].push_back(e); continue; }
        const double aA = std::atan2(ay[j] - y, ax[j] - x), aB = std::atan2(by[j] - y, bx[j] - x);
        double dl = aB - aA;
        while (dl > M_PI) dl -= two_pi;
        while (dl <= -M_PI) dl += two_pi;
        const double a0 = dl >= 0 ? aA : aB, span = std::fabs(dl);
        const double wid = std::asin(std::min(1.0, R / d)) + 2e-3;
        const long k0 = (long)std::floor((a0 - wid) / dbin), k1 = (long)std::floor((a0 + span + wid) / dbin);
        if (k1 - k0 + 1 >= BEAM_NB) { for (int k = 0; k < BEAM_NB; ++k) L[k].push_back(e); continue; }
        for (long k = k0; k <= k1; ++k) L[((k % BEAM_NB) + BEAM_NB) % BEAM_NB].push_back(e);
      }
      for (int k = 0; k < BEAM_NB; ++k) std::sort(L[k].begin(), L[k].end());
    }
  };
  const int nth = std::max(1, std::min(16, (int)std::thread::hardware_concurrency()));
  std::vector<std::thread> th;
  for (int k = 0; k < nth; ++k) th.emplace_back(work, (int)((long)ncell * k / nth), (int)((long)ncell * (k + 1) / nth));
  for (auto& x : th) x.join();
  // 16-bit entries: the bound code c = floor(sqrt(bound / kq)), so c^2 kq <= the wall's bound (rounded down again where
  // the double sqrt rounded up onto an integer), at most cmax - 1; each list sorted by entry, so the codes ascend
  const uint32_t cmax = B.g.cmax;
  const double kq = (double)B.g.kq;
  auto code_of = [&](uint32_t e) {
    const double lb = (double)(e >> 16) * 0.01;   // the cm bound, itself rounded down
    int c = (int)std::min<double>((double)cmax - 1.0, std::floor(std::sqrt(lb / kq)));
    while (c > 0 && (double)(c * c) * kq > lb) --c;
    return (uint16_t)(((uint32_t)c << wb) | (e & 0xFFFFu));
  };
  // per list (cell-major, slot order, beam_slot): the head record holds its first BEAM_HEAD entries (BEAM_PAD filled)
  // and, when the list is longer, 1 + the offset of its continuation -- the remaining entries followed by one BEAM_PAD
  // sentinel, so a walk needs no list end -- from its chunk's first ent[] index.  ent[0] is a sentinel; BEAM_COOP_PAD
  // sentinels close the array (the chunked and the wave-cooperative walks read past a list's sentinel).  A cell whose
  // continuations would overflow its chunk's 16-bit offsets keeps no lists (its rays take the wall-group walk).
  B.nxc = (nx + BEAM_CHUNK - 1) / BEAM_CHUNK;
  B.chunk.assign((size_t)B.nxc * ny, make_int4(-1, 0, 0, 0));
  std::vector<uint8_t> keep(ncell, 1);
  B.dropped = 0;
  for (int c0 = 0, c1; c0 < ncell; c0 = c1) {   // cells of one chunk: consecutive in row-major order
    const int key = cells[c0] / nx * B.nxc + cells[c0] % nx / BEAM_CHUNK;
    for (c1 = c0; c1 < ncell && cells[c1] / nx * B.nxc + cells[c1] % nx / BEAM_CHUNK == key; ++c1) {}
    size_t used = 0;
    for (int ci = c0; ci < c1; ++ci) {
      size_t cont = 0;
      for (int slot = 0; slot < BEAM_NB; ++slot) {
        const size_t len = lists[(size_t)ci * BEAM_NB + slot].size();
        if (len > (size_t)BEAM_HEAD) cont += len - BEAM_HEAD + 1;
      }
      if (used + cont >= BEAM_CONT_MAX) { keep[ci] = 0; ++B.dropped; } else used += cont;
    }
  }
  const size_t nkept = (size_t)ncell - B.dropped, nlist = nkept * BEAM_NB;
  B.head.assign(nlist, make_uint2(BEAM_PAD | (BEAM_PAD << 16), BEAM_PAD));
  B.ent.assign(1, (uint16_t)BEAM_PAD);
  B.entries = 0;
  std::vector<uint16_t> L16;
  int id = 0, cur = -1;
  size_t cb = 0;
  for (int ci = 0; ci < ncell; ++ci) {
    if (!keep[ci]) continue;
    const int cx = cells[ci] % nx, cy = cells[ci] / nx, key = cy * B.nxc + cx / BEAM_CHUNK;
    int4& ch = B.chunk[key];
    if (key != cur) { cur = key; cb = B.ent.size(); ch = make_int4(id * BEAM_NB, (int)cb, 0, 0); }
    ch.z = (int)((uint32_t)ch.z | (1u << (cx % BEAM_CHUNK)));
    for (int slot = 0; slot < BEAM_NB; ++slot) {
      const auto& L = lists[(size_t)ci * BEAM_NB + beam_bin(slot)];
      B.entries += L.size();
      L16.resize(L.size());
      for (size_t k = 0; k < L.size(); ++k) L16[k] = code_of(L[k]);
      std::sort(L16.begin(), L16.end());
      uint32_t h[4];
      for (int k = 0; k < BEAM_HEAD; ++k) h[k] = (size_t)k < L16.size() ? L16[k] : BEAM_PAD;
      h[3] = 0u;
      if (L16.size() > (size_t)BEAM_HEAD) {
        h[3] = (uint32_t)(B.ent.size() - cb) + 1u;
        B.ent.insert(B.ent.end(), L16.begin() + BEAM_HEAD, L16.end());
        B.ent.push_back((uint16_t)BEAM_PAD);
      }
      B.head[(size_t)id * BEAM_NB + slot] = make_uint2(h[0] | (h[1] << 16), h[2] | (h[3] << 16));
    }
    ++id;
  }
  for (int k = 0; k < (RAY_CHUNK > BEAM_COOP_PAD ? RAY_CHUNK : BEAM_COOP_PAD); ++k) B.ent.push_back((uint16_t)BEAM_PAD);
  if (getenv("NASCAR_VERBOSE"))
    fprintf(stderr, "build_beams: %d walls (%u-bit wall indices, bound codes of %.4f m x c^2), %d cells with lists, %zu "
            "dropped (continuation offsets), %zu entries, heads %.1f MB + continuations %.1f MB\n", nw, B.g.wbits,
            (double)B.g.kq, ncell - (int)B.dropped, B.dropped, B.entries, 8.0 * B.head.size() / 1e6, 2.0 * B.ent.size() / 1e6);
  B.nlist = nlist;
  B.build_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}
static int upload_beams(HostTrack& t) {
  auto& B = t.beam;
  if (B.ent.size() >= 0x7FFFFFF0u) return fail("beam list continuations hold %zu entries (31-bit cell offsets)", B.ent.size());
  HIPCHK(hipMalloc(&B.d_chunk, sizeof(int4) * std::max<size_t>(B.chunk.size(), 1)));
  if (!B.chunk.empty()) HIPCHK(hipMemcpy(B.d_chunk, B.chunk.data(), sizeof(int4) * B.chunk.size(), hipMemcpyHostToDevice));
  HIPCHK(hipMalloc(&B.d_ent, sizeof(uint16_t) * std::max<size_t>(B.ent.size(), 1)));
  if (!B.ent.empty()) HIPCHK(hipMemcpy(B.d_ent, B.ent.data(), sizeof(uint16_t) * B.ent.size(), hipMemcpyHostToDevice));
  HIPCHK(hipMalloc(&B.d_head, sizeof(uint2) * std::max<size_t>(B.head.size(), 1)));
  if (!B.head.empty()) HIPCHK(hipMemcpy(B.d_head, B.head.data(), sizeof(uint2) * B.head.size(), hipMemcpyHostToDevice));
  B.g.chunk = B.d_chunk; B.g.nxc = B.nxc; B.g.ent = B.d_ent; B.g.head = B.d_head;
  return 0;
}

static int upload_grid(HostGrid& G) {
  HIPCHK(hipMalloc(&G.d_start, sizeof(int) * G.start.size()));
  HIPCHK(hipMemcpy(G.d_start, G.start.data(), sizeof(int) * G.start.size(), hipMemcpyHostToDevice));
  HIPCHK(hipMalloc(&G.d_idx, sizeof(uint16_t) * std::max<size_t>(G.idx.size(), 1)));
  if (!G.idx.empty()) HIPCHK(hipMemcpy(G.d_idx, G.idx.data(), sizeof(uint16_t) * G.idx.size(), hipMemcpyHostToDevice));
  G.g.start = G.d_start; G.g.idx = G.d_idx; G.g.box = nullptr;
  if (!G.box.empty()) {
    HIPCHK(hipMalloc(&G.d_box, sizeof(float4) * G.box.size()));
    HIPCHK(hipMemcpy(G.d_box, G.box.data(), sizeof(float4) * G.box.size(), hipMemcpyHostToDevice));
    G.g.box = G.d_box;
  }
  return 0;
}

// A built track: the device tables of one .track (walls, segments, grids, beam lists, sensor image), read-only
// once built.  Handles share them through a process-wide cache keyed by the track's input arrays and the device:
// every env of a batch, every VecEnv sub-engine and every later handle on the same track uses one copy (the beam
// lists are 0.2-0.5 GB per track at 1 m cells and take ~2 s of host time to build).  The last handle to drop a
// build frees its device memory.
struct TrackBuild {
  int device = 0;
  HostTrack t;
  size_t lds = 0;   // model_kernel's LDS wall table
  ~TrackBuild() {
    int cur = 0;
    hipGetDevice(&cur);
    if (cur != device) hipSetDevice(device);
    hipFree(t.d_walls); hipFree(t.d_wfat); hipFree(t.d_segs); hipFree(t.d_prefix);
    hipFree(t.bp.d_start); hipFree(t.bp.d_idx); hipFree(t.bp.d_box); hipFree(t.sn.d_start); hipFree(t.sn.d_idx);
    hipFree(t.d_groups); hipFree(t.d_swall);
    hipFree(t.beam.d_chunk); hipFree(t.beam.d_ent); hipFree(t.beam.d_head);
    if (cur != device) hipSetDevice(cur);
  }
};
static std::mutex g_track_mu;
static std::unordered_map<std::string, std::weak_ptr<TrackBuild>> g_track_cache;

struct NascarHandle {
  NascarConfig cfg;
  int N, E, C, epb;
  void* arena = nullptr; size_t arena_bytes = 0;
  size_t off_f32, off_f64, off_i32, off_acc, off_ct, off_key, off_n, off_time, off_ei32, off_ctl;
  std::vector<std::shared_ptr<TrackBuild>> tracks;   // shared, read-only track tables (track_cache)
  TrackDev* d_tracks = nullptr;
  int* d_blk_track = nullptr; int* d_blk_env = nullptr; int nblocks = 0;
  int map_identity = 0, one_track = -1;   // Params shortcuts of the block map (prepare)
  std::vector<int> env_track;
  std::vector<int> pending_track;   // nascar_set_env_tracks, applied per env by its next nascar_reset
  bool pristine = true;             // no reset / step / rollout / set_state yet: track changes apply at once
  int car_contact = 0;              // nascar_set_car_contact (build-only extension)
  int ray_lanes = 0;                // nascar_set_sensor_lanes: 0 automatic, 4 or 16 lanes per car
  // threads per ray_sensor_kernel workgroup at 16 lanes per car (nascar_set_sensor_block).  64 / 128: the walks read
  // the track's wall image from global memory (L2-resident); the workgroups need no LDS, so they start on any CU with
  // free wave slots, beside the other shards' step workgroups (which hold ~52 KiB of LDS each).  256 / 512 / 1024:
  // every workgroup stages the whole image in LDS (larger ones stage it once for more cars).  Round 5 (per-shard
  // sensor dispatch at the steady state, 2 rounds): 64 21.0 / 20.9, 128 21.1 / 20.9, 256 (global walls) 23.5 / 23.5,
  // 512 (global) 25.9 / 26.1, 512 (LDS) 25.9 / 25.9 us; driver's command 128 131.6 / 132.2 vs 512 (LDS) 136.7 / 134.9
  // us per step.  Round 4 (LDS, driver's command): 256 151.9 / 150.3, 512 147.3 / 147.9, 1024 151.4 / 154.4
  int sensor_block = 128;
  int fuse_ml = 1;                  // nascar_set_fused_logic: model_logic_kernel (default) or model_kernel + logic_kernel
  float beam_cell = BEAM_CELL_M;    // nascar_set_beam_cell: cell size (m) of the beam lists of tracks added later
  float* d_vhist = nullptr;  // [VH_RING][N] speed history (nascar_set_perf_history), outside the snapshot arena
  double* d_ctl = nullptr;   // rule-driver state for nascar_policy_actions (inside the arena: snapshots keep it)
  float4* d_pose = nullptr;  // [2][N] step/reset -> sensor_kernel hand-off
  double2* d_pose_cs = nullptr;
  double2* d_ray_cs = nullptr;
  void* d_actor = nullptr;   // SAC actor weights (nascar_set_actor), one allocation
  void* d_params = nullptr;  // device copy of the launch Params (rollout_kernel) and the host image last uploaded
  Params params_up; bool params_valid = false;
  ActorDev actor{};
  void* d_actor32 = nullptr; ActorF32 actor32{};   // fp32 copies (nascar_set_actor_precision)
  int actor_fp32 = 1;   // default: reference precision
  size_t max_lds = 0, max_sensor_lds = 0, max_sensor_groups_lds = 0;
  bool dirty_tracks = true;
  // sharded rollout (nascar_set_rollout_streams): shard s steps workgroups [nblocks*s/S, nblocks*(s+1)/S) on its
  // own stream; the caller's stream forks to them at the launch and joins them at its end
  int ro_streams = 4;               // nascar_create: min(4, the process's hardware queues GPU_MAX_HW_QUEUES)
  std::vector<hipStream_t> sub_stream;
  hipEvent_t ev_fork = nullptr;
  std::vector<hipEvent_t> ev_join;
  float* d_ro_act = nullptr;        // [N][2] actions of a policy-2 (SAC actor) sharded rollout
  // pipelined rollout (nascar_set_rollout_pipe): sensor workgroups of pipe_sensor_kernel (0: off), the item ring,
  // counters (claimed, published, sticky error, pad) and per-workgroup completion counts
  int ro_pipe = 0;
  unsigned long long* d_pipe_ring = nullptr; size_t pipe_cap = 0;
  unsigned* d_pipe_ctr = nullptr; unsigned* d_pipe_sdone = nullptr; size_t pipe_nb = 0;
  unsigned pipe_seq = 0;
  hipEvent_t step_ev[4] = {nullptr, nullptr, nullptr, nullptr};   // nascar_set_step_events (profiling)
  // prepare(): capacities of the track table / block map buffers, pinned staging of their stream-ordered uploads
  size_t cap_tracks = 0, cap_blocks = 0, cap_blk_env = 0;
  void* h_stage = nullptr; size_t stage_bytes = 0;
  hipEvent_t ev_stage = nullptr;
  // random-track mode (nascar_set_random_tracks): the env -> track map, draw counters and seeds live on the device and
  // the block map is rebuilt there (block_map_kernel) after every launch that may change a track -- no host round trip
  int rt_on = 0, rt_ntracks = 0;
  void* d_rt = nullptr;             // one allocation: the arrays below
  int* d_rt_env_track = nullptr; int* d_rt_draws = nullptr; uint64_t* d_rt_seed = nullptr; int* d_rt_tracks = nullptr;
  int* d_rt_dirty = nullptr; uint8_t* d_rt_flags = nullptr;   // flags: env flags of a step whose caller passed none
};

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

extern "C" const char* nascar_last_error(void) { return g_err.c_str(); }

// envs per workgroup of the one-lane-per-car kernels: as many whole envs as fit (SBLOCK / C), unless that leaves
// fewer than 2 workgroups per CU -- a small batch (e.g. 4096 envs x 1 car: 32 workgroups) is then spread over
// 2 x CUs workgroups with fewer envs each.  Every step kernel lasts as long as its slowest wave, and a wave's
// time is the sum over its phases of the slowest lane's: fewer cars per wave shorten the slowest car's wait on
// its wave-mates (the chip has room for the extra, partly empty waves).  nascar_set_envs_per_block overrides it
// (and, in tools builds with -DNASCAR_AB_KNOBS only, NASCAR_EPB).
static int auto_epb(int E, int C, int device) {
  int epb = SBLOCK / C;
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0) cus = 256;
  const long target = 2L * cus;
  if ((E + epb - 1) / epb < target) epb = std::max(1, (int)((E + target - 1) / target));
#ifdef NASCAR_AB_KNOBS   // A/B tools builds only: the product library reads no environment knob that changes a kernel path
  if (const char* ev = getenv("NASCAR_EPB")) { const int v = atoi(ev); if (v >= 1 && v <= SBLOCK / C) epb = v; }
#endif
  return epb;
}

// Layout of the envs over the step kernels' workgroups (a scheduling choice: every env's state lives in the
// env-indexed arena whatever its workgroup, so results do not depend on it; tests pin that against the oracle).
extern "C" int nascar_set_envs_per_block(NascarHandle* h, int32_t epb) {
  if (!h) return fail("null argument");
  const int mx = SBLOCK / h->C;
  if (epb == 0) epb = auto_epb(h->E, h->C, h->cfg.device);
  if (epb < 1 || epb > mx) return fail("envs per workgroup must be in [1, %d] for %d cars per env (0: automatic), got %d",
                                      mx, h->C, epb);
  if (epb != h->epb) { h->epb = epb; h->dirty_tracks = true; }   // prepare() rebuilds the block map
  return 0;
}
extern "C" int nascar_get_envs_per_block(NascarHandle* h) { return h ? h->epb : -1; }
extern "C" int nascar_set_fused_logic(NascarHandle* h, int32_t enable) {
  if (!h) return fail("null argument");
  h->fuse_ml = enable != 0;
  return 0;
}
extern "C" int nascar_get_fused_logic(NascarHandle* h) { return h ? h->fuse_ml : -1; }
extern "C" int nascar_set_beam_cell(NascarHandle* h, float meters) {
  if (!h) return fail("null argument");
  if (!(meters >= BEAM_CELL_MIN && meters <= BEAM_CELL_MAX))
    return fail("beam cell size must be in [%.1f, %.1f] m, got %g", (double)BEAM_CELL_MIN, (double)BEAM_CELL_MAX, (double)meters);
  h->beam_cell = meters;
  return 0;
}
extern "C" int nascar_set_sensor_block(NascarHandle* h, int32_t threads) {
  if (!h) return fail("null argument");
  if (threads != 0 && threads != 64 && threads != 128 && threads != 256 && threads != 512 && threads != 1024)
    return fail("sensor workgroup size must be 0 (automatic: 128), 64, 128, 256, 512 or 1024 threads, got %d", threads);
  h->sensor_block = threads ? threads : 128;
  return 0;
}
extern "C" int nascar_set_sensor_lanes(NascarHandle* h, int32_t lanes) {
  if (!h) return fail("null argument");
  if (lanes != 0 && lanes != 4 && lanes != 16) return fail("sensor lanes per car must be 0 (automatic), 4 or 16, got %d", lanes);
  h->ray_lanes = lanes;
  return 0;
}

extern "C" int nascar_create(const NascarConfig* cfg, NascarHandle** out) {
  if (!cfg || !out) return fail("null argument");
  if (cfg->num_envs < 1) return fail("num_envs must be >= 1");
  if (cfg->num_cars < 1 || cfg->num_cars > 64) return fail("num_cars must be in [1, 64]");
  HIPCHK(hipSetDevice(cfg->device));
  NascarHandle* h = new NascarHandle();
  h->cfg = *cfg;
  h->E = cfg->num_envs; h->C = cfg->num_cars; h->N = h->E * h->C;
  h->epb = auto_epb(h->E, h->C, cfg->device);
#ifdef NASCAR_AB_KNOBS   // A/B tools builds only (the product library: nascar_set_sensor_lanes / _fused_logic /
                         // _sensor_block / _beam_cell)
  if (const char* ev = getenv("NASCAR_RAY_LPC")) h->ray_lanes = atoi(ev);
  if (const char* ev = getenv("NASCAR_FUSE_ML")) h->fuse_ml = atoi(ev) != 0;
  if (const char* ev = getenv("NASCAR_RBLOCK")) {
    const int rb = atoi(ev);
    if (rb == 64 || rb == 128 || rb == 256 || rb == 512 || rb == 1024) h->sensor_block = rb;
  }
  if (const char* ev = getenv("NASCAR_BEAM_CELL")) {
    const float v = (float)atof(ev);
    if (v >= BEAM_CELL_MIN && v <= BEAM_CELL_MAX) h->beam_cell = v;
  }
#endif
  size_t N = h->N, E = h->E, o = 0;
  h->off_f32 = o; o = align256(o + sizeof(float) * N_F32 * N);
  h->off_f64 = o; o = align256(o + sizeof(double) * N_F64 * N);
  h->off_i32 = o; o = align256(o + sizeof(int) * N_I32 * N);
  h->off_acc = o; o = align256(o + sizeof(double) * 20 * N);
  h->off_ct = o; o = align256(o + sizeof(DContact) * MAXC * N);
  h->off_key = o; o = align256(o + sizeof(int) * MAXC * N);
  h->off_n = o; o = align256(o + sizeof(float) * 2 * MAXC * N);
  h->off_time = o; o = align256(o + sizeof(double) * E);
  h->off_ei32 = o; o = align256(o + sizeof(int) * N_EI32 * E);
  h->off_ctl = o; o = align256(o + sizeof(double) * 4 * N);
  h->arena_bytes = o;
  hipError_t e = hipMalloc(&h->arena, o);
  if (e != hipSuccess) { delete h; return fail("hipMalloc(%zu) failed: %s", o, hipGetErrorString(e)); }
  hipMemset(h->arena, 0, o);
  h->d_ctl = (double*)((char*)h->arena + h->off_ctl);
  // pose hand-off [2][N] float4, then the per-env reset bytes (Params::reset_env)
  const size_t pose_bytes = sizeof(float4) * 2 * N + ((size_t)E + 15) / 16 * 16;
  if (hipMalloc(&h->d_pose, pose_bytes) != hipSuccess) { hipFree(h->arena); delete h; return fail("hipMalloc(pose) failed"); }
  hipMemset(h->d_pose, 0, pose_bytes);
  if (hipMalloc(&h->d_pose_cs, sizeof(double2) * 2 * N) != hipSuccess) { hipFree(h->arena); hipFree(h->d_pose); delete h; return fail("hipMalloc(pose_cs) failed"); }
  hipMemset(h->d_pose_cs, 0, sizeof(double2) * 2 * N);
  HIPCHK(hipMalloc(&h->d_ray_cs, sizeof(h_ray_cs)));
  HIPCHK(hipMemcpy(h->d_ray_cs, h_ray_cs, sizeof(h_ray_cs), hipMemcpyHostToDevice));
  h->env_track.assign(E, 0);
  {   // 4 shards, fewer if the process has fewer hardware queues (two shards on one queue run back to back);
      // more than 4 measured slower even with as many queues (tools/ro_queues_ab.sh: 6 / 8 / 12 shards on 6 / 8 / 12
      // queues 0.275 / 0.276 / 0.350 ms per step vs 0.193 ms for 4)
    const char* q = getenv("GPU_MAX_HW_QUEUES");
    const int nq = q ? atoi(q) : 4;
    h->ro_streams = std::max(1, std::min(nq > 0 ? nq : 4, 4));
  }
  *out = h;
  return 0;
}

extern "C" void nascar_destroy(NascarHandle* h) {
  if (!h) return;
  hipFree(h->d_vhist);
  hipFree(h->arena); hipFree(h->d_pose); hipFree(h->d_pose_cs); hipFree(h->d_ray_cs); hipFree(h->d_actor); hipFree(h->d_actor32); hipFree(h->d_params);
  hipFree(h->d_pipe_ring); hipFree(h->d_pipe_ctr); hipFree(h->d_pipe_sdone);
  {   // the shared track builds are released (and freed by the last holder) under the cache lock
    std::lock_guard<std::mutex> lk(g_track_mu);
    h->tracks.clear();
  }
  hipFree(h->d_tracks); hipFree(h->d_blk_track); hipFree(h->d_blk_env);
  if (h->ev_stage) { hipEventSynchronize(h->ev_stage); hipEventDestroy(h->ev_stage); }
  if (h->h_stage) hipHostFree(h->h_stage);
  for (auto st : h->sub_stream) hipStreamDestroy(st);
  for (auto ev : h->ev_join) hipEventDestroy(ev);
  if (h->ev_fork) hipEventDestroy(h->ev_fork);
  hipFree(h->d_ro_act);
  hipFree(h->d_rt);
  delete h;
}

static int sensor_lds_reserve(size_t need);
static int host_track(HostTrack& t, const std::string& key, const double* segments, int32_t nseg, double total_length,
                      const double* walls, int32_t nwall, float beam_cell, int* loaded = nullptr);
static std::string track_key(const double* segments, int32_t nseg, double total_length, const double* walls,
                             int32_t nwall, float beam_cell);
static int upload_track(HostTrack& t, size_t& lds_out);
static void retain_build(const std::shared_ptr<TrackBuild>& tb);
// wall table exactly as Box2D sees it (float32 transform via glibc sinf/cosf, fat AABB, key)
extern "C" int nascar_add_track(NascarHandle* h, const double* segments, int32_t nseg, double total_length,
                                const double* walls, int32_t nwall) {
  if (!h || !segments || !walls) return fail("null argument");
  if (nseg < 1 || nseg > MAX_SEG) return fail("segment count %d out of range", nseg);
  if (nwall < 1) return fail("track has no walls");
  const std::string dkey = track_key(segments, nseg, total_length, walls, nwall, h->beam_cell);   // (disk cache key)
  const std::string key = std::string((const char*)&h->cfg.device, sizeof h->cfg.device) + dkey;
  std::lock_guard<std::mutex> lk(g_track_mu);
  std::shared_ptr<TrackBuild> tb;
  {
    auto it = g_track_cache.find(key);
    if (it != g_track_cache.end()) tb = it->second.lock();
  }
  if (!tb) {
    tb = std::make_shared<TrackBuild>();
    tb->device = h->cfg.device;
    int cur = 0;
    HIPCHK(hipGetDevice(&cur));
    if (cur != h->cfg.device) HIPCHK(hipSetDevice(h->cfg.device));
    int rc = host_track(tb->t, dkey, segments, nseg, total_length, walls, nwall, h->beam_cell);
    if (rc == 0) rc = upload_track(tb->t, tb->lds);
    if (cur != h->cfg.device) hipSetDevice(cur);
    if (rc < 0) return rc;
    g_track_cache[key] = tb;
  }
  retain_build(tb);
  const HostTrack& t = tb->t;
  const size_t need = 2 * sizeof(float4) * t.walls.size() + sizeof(float4) * t.groups.size();
  if (need > h->max_sensor_lds) {   // on the handle's device (the attribute is per device), cached track or not
    int cur = 0;
    HIPCHK(hipGetDevice(&cur));
    if (cur != h->cfg.device) HIPCHK(hipSetDevice(h->cfg.device));
    const int rc = sensor_lds_reserve(need);
    if (cur != h->cfg.device) hipSetDevice(cur);
    if (rc < 0) return rc;
  }
  h->max_sensor_lds = std::max(h->max_sensor_lds, need);
  h->max_sensor_groups_lds = std::max(h->max_sensor_groups_lds, sizeof(float4) * t.groups.size());
  h->max_lds = std::max(h->max_lds, tb->lds);
  h->tracks.push_back(tb);
  h->dirty_tracks = true;
  return (int)h->tracks.size() - 1;
}

// The sensor wall image (2 float4 per wall + 1 per wall group) lives in the dynamic LDS of the kernels that stage it
// (ray_sensor_kernel, the fused rollout_kernel); with their static LDS it must fit the CU's 160 KiB, so that bounds
// the walls a track may have (~4 000 with the fused rollout's static LDS, ~4 900 for the sensor kernel alone; the
// bundled tracks have 730-732).  Images beyond 64 KiB are declared to the runtime first.
static int sensor_lds_reserve(size_t need) {
  const void* kern[] = {(const void*)ray_sensor_kernel<4>, (const void*)ray_sensor_kernel<16>,
                        (const void*)ray_sensor_kernel<16, 512>, (const void*)ray_sensor_kernel<16, 1024>,
                        (const void*)rollout_kernel};
  for (const void* k : kern) {
    hipFuncAttributes a;
    if (hipFuncGetAttributes(&a, k) != hipSuccess) return fail("hipFuncGetAttributes failed");
    // the fused rollout kernel also holds the car-car extension's scratch after the wall image
    const size_t n2 = k == (const void*)rollout_kernel ? ((need + 15) & ~(size_t)15) + CC_LDS_BYTES : need;
    if (a.sharedSizeBytes + n2 > LDS_PER_CU)
      return fail("track needs %zu B of LDS for its sensor wall image; with %zu B of static LDS a workgroup has %zu",
                  need, (size_t)a.sharedSizeBytes, LDS_PER_CU - (size_t)a.sharedSizeBytes);
    if (n2 > 64 * 1024) HIPCHK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)n2));
  }
  return 0;
}
// the host tables of one track (nascar_add_track): walls as Box2D sees them, segments, grids, beam lists, wall groups
static int host_build_track(HostTrack& t, const double* segments, int32_t nseg, double total_length,
                            const double* walls, int32_t nwall, float beam_cell) {
  t.total_length = total_length;
  t.startline = -1; t.has_banking = 0;
  double pre = 0.0;
  for (int k = 0; k < nseg; ++k) {
    const double* s = segments + 13 * k;
    DSeg d;
    d.sx = s[2]; d.sy = s[3]; d.ex = s[4]; d.ey = s[5]; d.width = s[6]; d.banking = s[12];
    double br = d.banking * (M_PI / 180.0);
    d.la = (1500.0 * 9.81) * sin(fabs(br)) * 0.3;     // src/car.py:527-533
    d.chord = sqrt(pow(d.ex - d.sx, 2.0) + pow(d.ey - d.sy, 2.0));
    t.prefix.push_back(pre);
    pre += d.chord;
    t.segs.push_back(d);
    if (t.startline < 0 && (int)s[0] == 1) t.startline = k;
    if (fabs(d.banking) >= 0.1) t.has_banking = 1;
  }
  std::unordered_map<std::string, int> keys;
  for (int j = 0; j < nwall; ++j) {
    const double* w = walls + 4 * j;
    HWall L;
    memset(&L, 0, sizeof L);
    L.px = (float)w[0]; L.py = (float)w[1]; L.ang = (float)w[2];
    L.qs = sinf(L.ang); L.qc = cosf(L.ang);
    L.hx = (float)w[3]; L.hy = (float)(1.0 / 2);
    L.rad = sqrtf(L.hx * L.hx + L.hy * L.hy) + 0.02f;
    float lx = 0, ly = 0, ux = 0, uy = 0;
    const float vx[4] = {-L.hx, L.hx, L.hx, -L.hx}, vy[4] = {-L.hy, -L.hy, L.hy, L.hy};
    for (int i = 0; i < 4; ++i) {
      float x = (L.qc * vx[i] - L.qs * vy[i]) + L.px;
      float y = (L.qs * vx[i] + L.qc * vy[i]) + L.py;
      if (i == 0) { lx = ux = x; ly = uy = y; }
      else { lx = x < lx ? x : lx; ly = y < ly ? y : ly; ux = ux > x ? ux : x; uy = uy > y ? uy : y; }
    }
    const float r = 2.0f * 0.005f;
    L.flx = (lx - r) - 0.1f; L.fly = (ly - r) - 0.1f; L.fhx = (ux + r) + 0.1f; L.fhy = (uy + r) + 0.1f;
    char kbuf[96];
    snprintf(kbuf, sizeof kbuf, "wall_%.1f_%.1f", (double)L.px, (double)L.py);
    auto it = keys.find(kbuf);
    if (it == keys.end()) { int id = (int)keys.size(); keys.emplace(kbuf, id); L.key = id; }
    else L.key = it->second;
    t.walls.push_back(L);
  }
  if (nwall > 65535) return fail("track has %d walls (grid and beam-list indices are 16-bit)", nwall);
  build_grids(t);
  build_beams(t, beam_cell);
  return 0;
}
// the device tables of a host-built (or cache-loaded) track, on the current device; lds: model_kernel's wall table bytes.
// The beam lists' host copies are released afterwards (the device copies are all the kernels use).
static int upload_track(HostTrack& t, size_t& lds_out) {
  {
    std::vector<LWall> dw(t.walls.begin(), t.walls.end());
    std::vector<float4> fat(t.walls.size());
    for (size_t j = 0; j < t.walls.size(); ++j) fat[j] = make_float4(t.walls[j].flx, t.walls[j].fly, t.walls[j].fhx, t.walls[j].fhy);
    HIPCHK(hipMalloc(&t.d_walls, sizeof(LWall) * dw.size()));
    HIPCHK(hipMemcpy(t.d_walls, dw.data(), sizeof(LWall) * dw.size(), hipMemcpyHostToDevice));
    HIPCHK(hipMalloc(&t.d_wfat, sizeof(float4) * fat.size()));
    HIPCHK(hipMemcpy(t.d_wfat, fat.data(), sizeof(float4) * fat.size(), hipMemcpyHostToDevice));
  }
  HIPCHK(hipMalloc(&t.d_segs, sizeof(DSeg) * t.segs.size()));
  HIPCHK(hipMemcpy(t.d_segs, t.segs.data(), sizeof(DSeg) * t.segs.size(), hipMemcpyHostToDevice));
  HIPCHK(hipMalloc(&t.d_prefix, sizeof(double) * t.prefix.size()));
  HIPCHK(hipMemcpy(t.d_prefix, t.prefix.data(), sizeof(double) * t.prefix.size(), hipMemcpyHostToDevice));
  if (upload_grid(t.bp) < 0 || upload_grid(t.sn) < 0) return -1;
  if (upload_beams(t) < 0) return -1;
  HIPCHK(hipMalloc(&t.d_groups, sizeof(float4) * t.groups.size()));
  HIPCHK(hipMemcpy(t.d_groups, t.groups.data(), sizeof(float4) * t.groups.size(), hipMemcpyHostToDevice));
  {   // the sensor kernel's wall image (same f32 values it would stage: rad + 0.25 rounded once)
    std::vector<float4> sw(2 * t.walls.size());
    for (size_t j = 0; j < t.walls.size(); ++j) {
      const HWall& w = t.walls[j];
      sw[2 * j] = make_float4(w.px, w.py, w.rad + 0.25f, w.hx);
      sw[2 * j + 1] = make_float4(w.qs, w.qc, w.hy, 0.0f);
    }
    HIPCHK(hipMalloc(&t.d_swall, sizeof(float4) * sw.size()));
    HIPCHK(hipMemcpy(t.d_swall, sw.data(), sizeof(float4) * sw.size(), hipMemcpyHostToDevice));
  }
  if (getenv("NASCAR_VERBOSE"))
    fprintf(stderr, "nascar_add_track: %zu walls, %zu groups; broadphase grid %dx%d (%zu entries), sensor grid %dx%d "
            "(%zu entries, mean %.1f per cell)\n", t.walls.size(), t.groups.size(), t.bp.g.nx, t.bp.g.ny, t.bp.idx.size(),
            t.sn.g.nx, t.sn.g.ny, t.sn.idx.size(), (double)t.sn.idx.size() / ((double)t.sn.g.nx * t.sn.g.ny));
  if (getenv("NASCAR_VERBOSE"))
    fprintf(stderr, "nascar_add_track: beam grid %dx%d (%.2f m cells), %zu cells with lists (%zu dropped: continuation "
            "offsets), %zu entries (mean %.2f per list), heads %.1f MB + continuations %.1f MB + cell chunks %.1f MB, built in "
            "%.2f s\n", t.beam.g.nx, t.beam.g.ny, 1.0 / (double)t.beam.g.inv_cell, t.beam.nlist / BEAM_NB,
            t.beam.dropped, t.beam.entries, (double)t.beam.entries / std::max<size_t>(1, t.beam.nlist),
            8.0 * t.beam.head.size() / 1e6, 2.0 * t.beam.ent.size() / 1e6, 16.0 * t.beam.chunk.size() / 1e6, t.beam.build_s);
  t.beam.chunk.clear(); t.beam.ent.clear(); t.beam.head.clear();
  t.beam.chunk.shrink_to_fit(); t.beam.ent.shrink_to_fit(); t.beam.head.shrink_to_fit();
  lds_out = sizeof(LWall) * t.walls.size();
  return 0;
}

// ------------------------------------------------------------------ track cache on disk (nascar_set_track_cache)
// A host build (walls, grids and 0.2-0.5 GB of beam lists per track at 1 m cells: ~2 s of 16 threads) written once and read
// by every later process: ranks of one node (bench.py --gpus N, learn/ppo.py-style SubprocVecEnv runs) share one build
// per track.  File = magic, format version, the full key (segments, walls, total length, cell size: compared byte for
// byte on load, so a hash collision can only miss), then the host tables.  Written to a temporary name and renamed; the
// builders of one key serialise on an flock'ed lock file, so concurrent ranks build each track once and the others load.
static const uint32_t TRACK_FILE_VERSION = 4;   // 4: 8-byte heads, 16-bit entries, per-track wall bits, chunked cell map
static std::string g_cache_dir;                       // "" = no disk cache (default)
static int g_retain = 8;                              // builds kept alive after their last handle (most recent first)
static std::deque<std::shared_ptr<TrackBuild>>* g_retained = new std::deque<std::shared_ptr<TrackBuild>>();
// (never destroyed: freeing device memory from a static destructor would run after the HIP runtime's own teardown)
static void retain_build(const std::shared_ptr<TrackBuild>& tb) {   // (g_track_mu held) most recently used first
  if (g_retain <= 0) return;
  auto& R = *g_retained;
  for (auto it = R.begin(); it != R.end(); ++it)
    if (*it == tb) { R.erase(it); break; }
  R.push_front(tb);
  while ((int)R.size() > g_retain) R.pop_back();
}

static uint64_t fnv1a64(const std::string& s, uint64_t h) {
  for (unsigned char c : s) { h ^= c; h *= 0x100000001B3ull; }
  return h;
}
struct Sink {
  FILE* f; bool ok = true;
  void raw(const void* p, size_t n) { if (ok && n && fwrite(p, 1, n, f) != n) ok = false; }
  template <class T> void pod(const T& v) { raw(&v, sizeof v); }
  template <class T> void vec(const std::vector<T>& v) { const uint64_t n = v.size(); pod(n); raw(v.data(), n * sizeof(T)); }
};
struct Source {
  FILE* f; bool ok = true;
  void raw(void* p, size_t n) { if (ok && n && fread(p, 1, n, f) != n) ok = false; }
  template <class T> void pod(T& v) { raw(&v, sizeof v); }
  template <class T> void vec(std::vector<T>& v) {
    uint64_t n = 0; pod(n);
    if (!ok || n > ((uint64_t)1 << 40) / sizeof(T)) { ok = false; return; }
    v.resize(n); raw(v.data(), n * sizeof(T));
  }
};
template <class IO, class HT> static void track_io(IO& io, HT& t) {   // the host tables, in file order
  io.vec(t.walls); io.vec(t.segs); io.vec(t.prefix);
  io.pod(t.total_length); io.pod(t.startline); io.pod(t.has_banking);
  io.pod(t.bp.g); io.vec(t.bp.start); io.vec(t.bp.idx); io.vec(t.bp.box);
  io.pod(t.sn.g); io.vec(t.sn.start); io.vec(t.sn.idx); io.vec(t.sn.box);
  io.pod(t.beam.g); io.vec(t.beam.chunk); io.pod(t.beam.nxc); io.vec(t.beam.ent); io.vec(t.beam.head);
  io.pod(t.beam.entries); io.pod(t.beam.nlist); io.pod(t.beam.dropped); io.pod(t.beam.build_s);
  io.vec(t.groups);
}
static bool load_track_file(const std::string& path, const std::string& key, HostTrack& t) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) return false;
  Source in{f};
  char magic[8] = {0}; uint32_t ver = 0; std::string k;
  in.raw(magic, 8); in.pod(ver);
  std::vector<char> kb; in.vec(kb);
  bool ok = in.ok && !memcmp(magic, "NASCARTK", 8) && ver == TRACK_FILE_VERSION && kb.size() == key.size() &&
            !memcmp(kb.data(), key.data(), key.size());
  if (ok) { track_io(in, t); ok = in.ok; }
  fclose(f);
  if (!ok) t = HostTrack();
  return ok;
}
static void save_track_file(const std::string& path, const std::string& key, HostTrack& t) {
  const std::string tmp = path + ".tmp." + std::to_string((long)getpid());
  FILE* f = fopen(tmp.c_str(), "wb");
  if (!f) return;                        // (a cache that cannot be written is only slower)
  Sink out{f};
  out.raw("NASCARTK", 8); out.pod(TRACK_FILE_VERSION);
  std::vector<char> kb(key.begin(), key.end()); out.vec(kb);
  track_io(out, t);
  const bool ok = out.ok && fclose(f) == 0;
  if (ok) rename(tmp.c_str(), path.c_str());
  else unlink(tmp.c_str());
}
// the track's inputs and the beam-list cell size (builds at different cell sizes differ): the disk cache's key
static std::string track_key(const double* segments, int32_t nseg, double total_length, const double* walls,
                             int32_t nwall, float beam_cell) {
  std::string k;
  const int32_t dims[2] = {nseg, nwall};
  k.append((const char*)dims, sizeof dims);
  k.append((const char*)&total_length, sizeof total_length);
  k.append((const char*)&beam_cell, sizeof beam_cell);
  k.append((const char*)segments, sizeof(double) * 13 * (size_t)nseg);
  k.append((const char*)walls, sizeof(double) * 4 * (size_t)nwall);
  return k;
}
// host tables of a track: from the disk cache when it holds this key (*loaded = 1), else built (and written there)
static int host_track(HostTrack& t, const std::string& key, const double* segments, int32_t nseg, double total_length,
                      const double* walls, int32_t nwall, float beam_cell, int* loaded) {
  if (loaded) *loaded = 0;
  if (g_cache_dir.empty()) return host_build_track(t, segments, nseg, total_length, walls, nwall, beam_cell);
  char name[64];
  snprintf(name, sizeof name, "track_%016llx%016llx.nbt", (unsigned long long)fnv1a64(key, 0xCBF29CE484222325ull),
           (unsigned long long)fnv1a64(key, 0x84222325CBF29CE4ull));
  const std::string path = g_cache_dir + "/" + name;
  if (load_track_file(path, key, t)) { if (loaded) *loaded = 1; return 0; }
  mkdir(g_cache_dir.c_str(), 0777);       // (one level; an existing directory is fine)
  const int lk = open((path + ".lock").c_str(), O_CREAT | O_RDWR, 0666);
  if (lk >= 0) flock(lk, LOCK_EX);       // another process may be building this key: wait for it, then load
  int rc = 0;
  if (lk >= 0 && load_track_file(path, key, t)) {
    if (loaded) *loaded = 1;
  } else {
    rc = host_build_track(t, segments, nseg, total_length, walls, nwall, beam_cell);
    if (rc == 0) save_track_file(path, key, t);
  }
  if (lk >= 0) { flock(lk, LOCK_UN); close(lk); }
  return rc;
}
// host only (no device): the track's tables into the disk cache -- loaded (returns 1) when a file for this key exists,
// else built and written (returns 0); a launcher prebuilds a job's tracks once before its ranks start
extern "C" int nascar_prebuild_track(const double* segments, int32_t nseg, double total_length, const double* walls,
                                     int32_t nwall, float beam_cell) {
  if (!segments || !walls) return fail("null argument");
  if (nseg < 1 || nseg > MAX_SEG) return fail("segment count %d out of range", nseg);
  if (nwall < 1) return fail("track has no walls");
  if (!(beam_cell >= BEAM_CELL_MIN && beam_cell <= BEAM_CELL_MAX))
    return fail("beam cell size must be in [%.1f, %.1f] m, got %g", (double)BEAM_CELL_MIN, (double)BEAM_CELL_MAX, (double)beam_cell);
  std::lock_guard<std::mutex> lk(g_track_mu);
  if (g_cache_dir.empty()) return fail("no track cache directory (nascar_set_track_cache)");
  HostTrack t;
  int loaded = 0;
  const int rc = host_track(t, track_key(segments, nseg, total_length, walls, nwall, beam_cell), segments, nseg,
                            total_length, walls, nwall, beam_cell, &loaded);
  return rc < 0 ? rc : loaded;
}
extern "C" int nascar_set_track_cache(int32_t retain, const char* dir) {
  if (retain < 0) return fail("retain must be >= 0, got %d", retain);
  std::lock_guard<std::mutex> lk(g_track_mu);
  g_retain = retain;
  while ((int)g_retained->size() > g_retain) g_retained->pop_back();
  g_cache_dir = dir ? dir : "";
  while (g_cache_dir.size() > 1 && g_cache_dir.back() == '/') g_cache_dir.pop_back();
  return 0;
}

extern "C" int nascar_set_env_tracks(NascarHandle* h, const int32_t* env_track) {
  if (!h || !env_track) return fail("null argument");
  for (int e = 0; e < h->E; ++e)
    if (env_track[e] < 0 || env_track[e] >= (int)h->tracks.size()) return fail("env %d: bad track id %d", e, env_track[e]);
  if (h->rt_on) return fail("random-track mode is on (nascar_set_random_tracks): the device draws every env's track");
  // recorded only: an env moves to its new track at its next nascar_reset, with fresh physics worlds (CarEnv.reset
  // recreates CarPhysics on a track change, src/car_env.py:375-394); until then it keeps stepping on its old track
  // (its Box2D contacts hold wall indices of that track)
  if (h->pristine) {   // nothing stepped or reset yet: no state on the old track, apply now
    h->env_track.assign(env_track, env_track + h->E);
    h->pending_track.clear();
    h->dirty_tracks = true;
    return 0;
  }
  h->pending_track.assign(env_track, env_track + h->E);
  return 0;
}

// nascar_reset's half of a track change: envs with a pending track that this reset covers switch now (E_CREATED
// cleared on the stream, so reset_kernel builds them fresh worlds); the block map is rebuilt by prepare()
static int apply_pending_tracks(NascarHandle* h, const uint8_t* env_mask, void* stream) {
  if (h->pending_track.empty()) return 0;
  bool any = false;
  for (int e = 0; e < h->E && !any; ++e) any = h->pending_track[e] != h->env_track[e];
  if (!any) { h->pending_track.clear(); return 0; }
  std::vector<uint8_t> mask(h->E, 1);
  if (env_mask) {   // device mask: one small synchronous copy, only when a track change is pending
    HIPCHK(hipMemcpyAsync(mask.data(), env_mask, h->E, hipMemcpyDeviceToHost, (hipStream_t)stream));
    HIPCHK(hipStreamSynchronize((hipStream_t)stream));
  }
  int* created = (int*)((char*)h->arena + h->off_ei32) + (size_t)E_CREATED * h->E;
  bool left = false;
  for (int e = 0; e < h->E; ++e) {
    if (h->pending_track[e] == h->env_track[e]) continue;
    if (!mask[e]) { left = true; continue; }
    h->env_track[e] = h->pending_track[e];
    HIPCHK(hipMemsetAsync(created + e, 0, sizeof(int), (hipStream_t)stream));
    h->dirty_tracks = true;
  }
  if (!left) h->pending_track.clear();
  return 0;
}

// Device copies of the track table and the block map, rebuilt when the env -> track assignment changed.
// Stream-ordered: the tables are uploaded with hipMemcpyAsync on the caller's stream, so the copies land after
// every earlier launch on that stream (the sharded rollout joins its shard streams into it before returning)
// and before every later one.  Buffers keep their capacity; only growth (the first call, a newly loaded track)
// reallocates, and then the old buffers are released after an explicit device synchronisation.  The host
// source is pinned staging memory owned by the handle, reused only after its previous upload has completed.
static int prepare(NascarHandle* h, hipStream_t stream) {
  if (h->tracks.empty()) return fail("no track loaded (nascar_add_track)");
  if (!h->dirty_tracks) return 0;
  std::vector<TrackDev> td;
  for (auto& tp : h->tracks) {
    const HostTrack& t = tp->t;
    TrackDev d;
    d.walls = t.d_walls; d.wfat = t.d_wfat; d.nwall = (int)t.walls.size(); d.segs = t.d_segs; d.nseg = (int)t.segs.size();
    d.prefix = t.d_prefix; d.total_length = t.total_length; d.startline = t.startline; d.has_banking = t.has_banking;
    d.bp = t.bp.g; d.sn = t.sn.g; d.groups = t.d_groups; d.ngroup = (int)t.groups.size(); d.swall = t.d_swall;
    d.beam = t.beam.g;
    td.push_back(d);
  }
  // workgroups hold whole envs of one track: group envs by track, pad each group to a block
  std::vector<int> blk_track, blk_env;
  if (h->rt_on) {   // random-track mode: the device builds the map (block_map_kernel) into a fixed grid of nb_cap blocks
    const size_t nt = td.size(), nb = (size_t)(h->E + h->epb - 1) / h->epb + nt;
    if (nt > RT_MAX_TRACKS) return fail("random-track mode supports at most %d loaded tracks", RT_MAX_TRACKS);
    if (nt > h->cap_tracks || nb > h->cap_blocks || nb * h->epb > h->cap_blk_env) {
      HIPCHK(hipDeviceSynchronize());
      if (nt > h->cap_tracks) {
        hipFree(h->d_tracks); h->d_tracks = nullptr;
        const size_t cap = std::max(nt, (size_t)8);
        HIPCHK(hipMalloc(&h->d_tracks, sizeof(TrackDev) * cap));
        h->cap_tracks = cap;
      }
      if (nb > h->cap_blocks || nb * h->epb > h->cap_blk_env) {
        hipFree(h->d_blk_track); hipFree(h->d_blk_env); h->d_blk_track = h->d_blk_env = nullptr;
        h->cap_blocks = h->cap_blk_env = 0;
        HIPCHK(hipMalloc(&h->d_blk_track, sizeof(int) * nb));
        HIPCHK(hipMalloc(&h->d_blk_env, sizeof(int) * nb * h->epb));
        h->cap_blocks = nb; h->cap_blk_env = nb * h->epb;
      }
    }
    const size_t b_tr = sizeof(TrackDev) * nt;
    if (h->ev_stage) HIPCHK(hipEventSynchronize(h->ev_stage));
    if (b_tr > h->stage_bytes) {
      if (h->h_stage) hipHostFree(h->h_stage);
      h->h_stage = nullptr; h->stage_bytes = 0;
      HIPCHK(hipHostMalloc(&h->h_stage, b_tr));
      h->stage_bytes = b_tr;
    }
    memcpy(h->h_stage, td.data(), b_tr);
    HIPCHK(hipMemcpyAsync(h->d_tracks, h->h_stage, b_tr, hipMemcpyHostToDevice, stream));
    if (!h->ev_stage) HIPCHK(hipEventCreateWithFlags(&h->ev_stage, hipEventDisableTiming));
    HIPCHK(hipEventRecord(h->ev_stage, stream));
    hipLaunchKernelGGL(block_map_kernel, dim3(1), dim3(1024), 0, stream, h->E, h->epb, (int)nt, h->d_rt_env_track,
                       h->d_blk_track, h->d_blk_env, (int)nb, h->d_rt_dirty, 1);
    HIPCHK(hipGetLastError());
    h->nblocks = (int)nb;
    h->map_identity = 0; h->one_track = -1;
    h->dirty_tracks = false;
    return 0;
  }
  // Each track's workgroups are spread evenly over the workgroup order (workgroup i of a track with n of them sorts at
  // (i + 1/2) / n): the sharded rollout cuts the order into contiguous shards, and with the tracks in id order one shard
  // held ~2 whole tracks of a mixed batch -- the shard with the tight tracks (more wall contacts and TOI events) set
  // every rollout call's length.  Interleaved, every shard gets its share of every track.  One track: the env order.
  {
    std::vector<std::vector<int>> per(h->tracks.size());
    for (int e = 0; e < h->E; ++e) per[h->env_track[e]].push_back(e);
    struct Blk { double key; int tr, i; };
    std::vector<Blk> order;
    for (int tr = 0; tr < (int)per.size(); ++tr) {
      const int nbt = (int)((per[tr].size() + h->epb - 1) / h->epb);
      for (int i = 0; i < nbt; ++i) order.push_back({(i + 0.5) / nbt, tr, i});
    }
    bool interleave = true;
#ifdef NASCAR_AB_KNOBS   // A/B tools builds only: NASCAR_MAP_CONTIGUOUS restores the round-5 track-major order
    if (getenv("NASCAR_MAP_CONTIGUOUS")) interleave = false;
#endif
    if (interleave)
      std::stable_sort(order.begin(), order.end(), [](const Blk& a, const Blk& b) { return a.key < b.key; });
    for (const Blk& b : order) {
      const std::vector<int>& envs = per[b.tr];
      blk_track.push_back(b.tr);
      for (int k = 0; k < h->epb; ++k) {
        const size_t j = (size_t)b.i * h->epb + k;
        blk_env.push_back(j < envs.size() ? envs[j] : -1);
      }
    }
  }
  const size_t nt = td.size(), nb = blk_track.size();
  // growth (a new track, a finer layout from nascar_set_envs_per_block): earlier launches may still read the old buffers
  if (nt > h->cap_tracks || nb > h->cap_blocks || blk_env.size() > h->cap_blk_env) {
    HIPCHK(hipDeviceSynchronize());
    if (nt > h->cap_tracks) {
      hipFree(h->d_tracks); h->d_tracks = nullptr;
      const size_t cap = std::max(nt, (size_t)8);
      HIPCHK(hipMalloc(&h->d_tracks, sizeof(TrackDev) * cap));
      h->cap_tracks = cap;
    }
    if (nb > h->cap_blocks || blk_env.size() > h->cap_blk_env) {
      hipFree(h->d_blk_track); hipFree(h->d_blk_env); h->d_blk_track = h->d_blk_env = nullptr;
      h->cap_blocks = h->cap_blk_env = 0;
      const size_t cap = std::max(nb, (size_t)(h->E + h->epb - 1) / h->epb + 8);
      const size_t cap_env = std::max(blk_env.size(), cap * h->epb);
      HIPCHK(hipMalloc(&h->d_blk_track, sizeof(int) * cap));
      HIPCHK(hipMalloc(&h->d_blk_env, sizeof(int) * cap_env));
      h->cap_blocks = cap; h->cap_blk_env = cap_env;
    }
  }
  const size_t b_tr = sizeof(TrackDev) * nt, b_bt = sizeof(int) * nb, b_be = sizeof(int) * blk_env.size();
  const size_t need = b_tr + b_bt + b_be;
  if (h->ev_stage) HIPCHK(hipEventSynchronize(h->ev_stage));   // the previous upload out of the staging buffer
  if (need > h->stage_bytes) {
    if (h->h_stage) hipHostFree(h->h_stage);
    h->h_stage = nullptr; h->stage_bytes = 0;
    HIPCHK(hipHostMalloc(&h->h_stage, need));
    h->stage_bytes = need;
  }
  char* st = (char*)h->h_stage;
  memcpy(st, td.data(), b_tr);
  memcpy(st + b_tr, blk_track.data(), b_bt);
  memcpy(st + b_tr + b_bt, blk_env.data(), b_be);
  HIPCHK(hipMemcpyAsync(h->d_tracks, st, b_tr, hipMemcpyHostToDevice, stream));
  HIPCHK(hipMemcpyAsync(h->d_blk_track, st + b_tr, b_bt, hipMemcpyHostToDevice, stream));
  HIPCHK(hipMemcpyAsync(h->d_blk_env, st + b_tr + b_bt, b_be, hipMemcpyHostToDevice, stream));
  if (!h->ev_stage) HIPCHK(hipEventCreateWithFlags(&h->ev_stage, hipEventDisableTiming));
  HIPCHK(hipEventRecord(h->ev_stage, stream));
  h->nblocks = (int)nb;
  h->map_identity = 1;
  for (size_t s = 0; s < blk_env.size(); ++s)
    if (blk_env[s] != ((int)s < h->E ? (int)s : -1)) { h->map_identity = 0; break; }
  h->one_track = blk_track.empty() ? -1 : blk_track[0];
  for (int tr : blk_track) if (tr != h->one_track) { h->one_track = -1; break; }
#ifdef NASCAR_AB_KNOBS
  if (getenv("NASCAR_NO_MAP_SHORTCUT")) { h->map_identity = 0; h->one_track = -1; }   // A/B tools builds only
#endif
  h->dirty_tracks = false;
  return 0;
}

static Params make_params(NascarHandle* h) {
  Params P;
  memset(&P, 0, sizeof P);   // padding too: nascar_rollout compares the bytes before re-uploading
  P.E = h->E; P.C = h->C; P.N = h->N; P.epb = h->epb; P.nblocks = h->nblocks; P.reset_on_lap = h->cfg.reset_on_lap;
  P.dt_d = 1.0 / 60.0; P.dt_f = (float)P.dt_d;
  P.friction = sqrtf(0.7f * 0.333f);
  P.start_x = h->cfg.start_x; P.start_y = h->cfg.start_y; P.start_angle = (float)h->cfg.start_angle;
  char* a = (char*)h->arena;
  P.f32 = (float*)(a + h->off_f32); P.f64 = (double*)(a + h->off_f64); P.i32 = (int*)(a + h->off_i32);
  P.acc = (double*)(a + h->off_acc); P.ct = (DContact*)(a + h->off_ct); P.act_key = (int*)(a + h->off_key);
  P.act_n = (float*)(a + h->off_n); P.env_time = (double*)(a + h->off_time); P.env_i32 = (int*)(a + h->off_ei32);
  P.blk_track = h->d_blk_track; P.blk_env = h->d_blk_env; P.tracks = h->d_tracks;
  P.map_identity = h->map_identity; P.one_track = h->one_track;
  P.pose = h->d_pose; P.reset_env = (uint8_t*)(h->d_pose + 2 * (size_t)h->N); P.pose_cs = h->d_pose_cs; P.ray_cs = h->d_ray_cs; P.ctl = h->d_ctl;
  P.vhist = h->d_vhist;
  P.car_contact = h->car_contact;
  return P;
}

// passes: 1 = pass A only (pose[n] with its A-mode bits: nascar_reset), 3 = pass A then pass B (the reset
// poses pose[N + n] of auto-reset cars overwrite those cars' pass-A obs values: nascar_step)
// the beam-list sensor kernel; tools builds with -DNASCAR_AB_KNOBS: NASCAR_SENSOR=groups selects the wall-group kernel
// for the step (the tests cross-check the two through nascar_debug_sensors)
static int sensor_impl() {
#ifdef NASCAR_AB_KNOBS
  static int m = -1;
  if (m < 0) { const char* e = getenv("NASCAR_SENSOR"); m = (e && !strcmp(e, "groups")) ? 0 : 1; }
  return m;
#else
  return 1;
#endif
}
// Lanes per car of the beam-list sensor kernel: one ray per lane (16 lanes per car) by default, so each car's four
// sequential walks (4 lanes per car: rays r, r + 4, r + 8, r + 12 per lane) become one and the kernel's slowest lane
// is one long walk instead of four.  Round 1 (4 m cells, whole-grid launches) measured 4 lanes faster at the
// headline's 81 920 cars (41.5 vs 62 us); with 1 m cells and the sharded rollout 16 lanes measure faster there too
// (driver's command 148.9 / 151.7 vs 158.0 / 155.2 us per step, round 4), as they did for small batches (cfg2).
// NASCAR_RAY_LPC = 4 / 16 or nascar_set_sensor_lanes overrides.
#ifndef RAY_LPC16_MAX_CARS
#define RAY_LPC16_MAX_CARS (1 << 30)
#endif
static int ray_lpc(const NascarHandle* h) {
  if (h->ray_lanes == 4 || h->ray_lanes == 16) return h->ray_lanes;   // nascar_set_sensor_lanes / NASCAR_RAY_LPC
  return h->N <= RAY_LPC16_MAX_CARS ? 16 : 4;
}
// nb step-kernel workgroups from P.blk0 (each is `sub` sensor workgroups)
static void launch_sensors_impl(NascarHandle* h, const Params& P, int nb, float* obs, float* terminal_obs, int passes,
                                void* stream, int impl) {
  if (impl == 1) {
    const size_t rlds = h->max_sensor_lds;   // >= 2 float4 per wall
    const int cars = h->epb * h->C;          // cars per step-kernel workgroup
    if (ray_lpc(h) == 16) {
      if (h->sensor_block < BLOCK) {   // 64 / 128 threads: the walls from the global image, no LDS
        const int rb = h->sensor_block, sub = (cars + rb / 16 - 1) / (rb / 16);
        if (rb == 64)
          hipLaunchKernelGGL((ray_sensor_kernel<16, 64, true>), dim3(nb * sub), dim3(rb), 0, (hipStream_t)stream, P, obs,
                             terminal_obs, passes, sub);
        else
          hipLaunchKernelGGL((ray_sensor_kernel<16, 128, true>), dim3(nb * sub), dim3(rb), 0, (hipStream_t)stream, P, obs,
                             terminal_obs, passes, sub);
        return;
      }
      // every sensor workgroup stages the whole wall image: larger workgroups stage it for more cars
      int rb = h->sensor_block;
      while (rb > BLOCK && rb / 2 >= cars * 16) rb /= 2;   // no wider than a step workgroup's cars need (small batches)
      const int sub = (cars + rb / 16 - 1) / (rb / 16);
      if (rb == 1024)
        hipLaunchKernelGGL((ray_sensor_kernel<16, 1024>), dim3(nb * sub), dim3(rb), rlds, (hipStream_t)stream, P, obs,
                           terminal_obs, passes, sub);
      else if (rb == 512)
        hipLaunchKernelGGL((ray_sensor_kernel<16, 512>), dim3(nb * sub), dim3(rb), rlds, (hipStream_t)stream, P, obs,
                           terminal_obs, passes, sub);
      else
        hipLaunchKernelGGL((ray_sensor_kernel<16, BLOCK>), dim3(nb * sub), dim3(BLOCK), rlds, (hipStream_t)stream, P, obs,
                           terminal_obs, passes, sub);
    } else {
      const int sub = (cars + BLOCK / RAY_LPC - 1) / (BLOCK / RAY_LPC);
      hipLaunchKernelGGL(ray_sensor_kernel<RAY_LPC>, dim3(nb * sub), dim3(BLOCK), rlds, (hipStream_t)stream, P, obs,
                         terminal_obs, passes, sub);
    }
    return;
  }
  const size_t lds = h->max_sensor_groups_lds;
  const int sub = (SBLOCK + BLOCK / SENSOR_LPC - 1) / (BLOCK / SENSOR_LPC);
  hipLaunchKernelGGL(sensor_kernel<SENSOR_LPC>, dim3(nb * sub), dim3(BLOCK), lds, (hipStream_t)stream,
                     P, obs, terminal_obs, passes);
}
static void launch_sensors(NascarHandle* h, const Params& P, float* obs, float* terminal_obs, int passes, void* stream) {
  launch_sensors_impl(h, P, h->nblocks, obs, terminal_obs, passes, stream, sensor_impl());
}

static RtDev rt_dev(const NascarHandle* h) {
  RtDev R;
  R.env_track = h->d_rt_env_track; R.draws = h->d_rt_draws; R.seed = h->d_rt_seed; R.tracks = h->d_rt_tracks;
  R.ntracks = h->rt_ntracks; R.dirty = h->d_rt_dirty;
  return R;
}
// the device-side block map rebuild (random-track mode): a no-op launch unless an env changed track since the last one
static int rt_block_map(NascarHandle* h, hipStream_t s, int force) {
  hipLaunchKernelGGL(block_map_kernel, dim3(1), dim3(1024), 0, s, h->E, h->epb, (int)h->tracks.size(), h->d_rt_env_track,
                     h->d_blk_track, h->d_blk_env, h->nblocks, h->d_rt_dirty, force);
  HIPCHK(hipGetLastError());
  return 0;
}
// random-track mode, after a step with auto-reset (env_flags: that step's, non-null): the reset envs draw their next
// tracks, the switching ones are reset there (rt_switch_kernel), and the block map follows
static int rt_after_step(NascarHandle* h, const Params& P, const uint8_t* env_flags, float* obs, hipStream_t s) {
  hipLaunchKernelGGL(rt_switch_kernel, dim3((h->E + 63) / 64), dim3(RT_SWITCH_BLOCK), 0, s, P, rt_dev(h), env_flags, obs);
  HIPCHK(hipGetLastError());
  return rt_block_map(h, s, 0);
}

extern "C" int nascar_reset(NascarHandle* h, const uint8_t* env_mask, float* obs, void* stream) {
  if (!h || !obs) return fail("null argument");
  h->pristine = false;
  if (!h->rt_on && apply_pending_tracks(h, env_mask, stream)) return -1;
  if (prepare(h, (hipStream_t)stream)) return -1;
  Params P = make_params(h);
  if (h->rt_on) {   // CarEnv.reset in random-track mode: a new track per reset env first (src/car_env.py:331-333)
    hipLaunchKernelGGL(rt_reset_draw_kernel, dim3((h->E + 255) / 256), dim3(256), 0, (hipStream_t)stream, P, rt_dev(h),
                       env_mask);
    HIPCHK(hipGetLastError());
    if (rt_block_map(h, (hipStream_t)stream, 0)) return -1;
  }
  hipLaunchKernelGGL(reset_kernel, dim3(h->nblocks), dim3(SBLOCK), 0, (hipStream_t)stream, P, env_mask, obs);
  HIPCHK(hipGetLastError());
  launch_sensors(h, P, obs, nullptr, 1, stream);
  HIPCHK(hipGetLastError());
  return 0;
}

static int step_impl(NascarHandle* h, const void* actions, int32_t discrete, int policy, uint64_t seed, int64_t step,
                     float* obs, float* reward, uint8_t* car_flags, uint8_t* env_flags, int32_t auto_reset,
                     float* terminal_obs, void* stream);
extern "C" int nascar_step(NascarHandle* h, const void* actions, int32_t discrete, float* obs, float* reward,
                           uint8_t* car_flags, uint8_t* env_flags, int32_t auto_reset, float* terminal_obs, void* stream) {
  if (!h || !actions || !obs || !reward) return fail("null argument");
  return step_impl(h, actions, discrete, -1, 0, 0, obs, reward, car_flags, env_flags, auto_reset, terminal_obs, stream);
}
extern "C" int nascar_step_driven(NascarHandle* h, int32_t policy, uint64_t seed, int64_t step, float* obs, float* reward,
                                  uint8_t* car_flags, uint8_t* env_flags, int32_t auto_reset, float* terminal_obs,
                                  void* stream) {
  if (!h || !obs || !reward) return fail("null argument");
  if (policy != 0 && policy != 1 && policy != 3) return fail("driven step policy must be 0, 1 or 3 (got %d)", policy);
  return step_impl(h, nullptr, 0, policy, seed, step, obs, reward, car_flags, env_flags, auto_reset, terminal_obs, stream);
}
// one env step of step-kernel workgroups [P.blk0, P.blk0 + nb) on stream s:
// model_kernel -> logic_kernel -> sensor_kernel (pass A for every car, pass B for auto-reset cars)
// obs_in: the observation the device driver reads (the previous step's); obs: where this step's is written
// phases: which of the three launches to enqueue (bit 0 model (+ car contact), bit 1 logic, bit 2 sensors), so
// the sharded rollout can enqueue one phase for every shard before the next phase (see rollout_sharded)
enum { PH_MODEL = 1, PH_LOGIC = 2, PH_SENSOR = 4, PH_ALL = 7 };
static int launch_step_range(NascarHandle* h, const Params& P, int nb, const void* actions, int32_t discrete, int policy,
                             uint64_t seed, int64_t step, const float* obs_in, float* obs, float* reward,
                             uint8_t* car_flags, uint8_t* env_flags, int32_t auto_reset, float* terminal_obs,
                             hipStream_t s, int phases = PH_ALL, bool model_issued = false) {
  const bool timed = h->step_ev[0] && nb == h->nblocks;   // nascar_set_step_events: whole-grid steps only
  if (h->fuse_ml && (CC_FUSED || !h->car_contact)) {   // model + logic in one launch (model_logic_kernel); logic is part of PH_MODEL
    // Under the fused kernel the logic phase IS part of PH_MODEL's launch, so a PH_LOGIC-only request enqueues nothing:
    // only a caller that has already requested PH_MODEL for the same step and range may make it (model_issued: the
    // sharded rollout's phase-major loop, 1 << ph for ph = 0, 1, 2); anyone else gets an error, not a silently
    // skipped env logic.  nascar_step / nascar_step_driven pass PH_ALL.
    if ((phases & PH_LOGIC) && !(phases & PH_MODEL) && !model_issued)
      return fail("the logic phase alone cannot run under the fused model + logic kernel (nascar_set_fused_logic(h, 0))");
    if (phases & PH_MODEL) {
      if (timed) HIPCHK(hipEventRecord(h->step_ev[0], s));
      hipLaunchKernelGGL(model_logic_kernel, dim3(nb), dim3(SBLOCK), MODEL_LOGIC_LDS_BYTES, s, P, actions, discrete,
                         terminal_obs != nullptr, policy, seed, step, obs_in, obs, reward, car_flags, env_flags, auto_reset,
                         terminal_obs);
      HIPCHK(hipGetLastError());
      if (timed) { HIPCHK(hipEventRecord(h->step_ev[1], s)); HIPCHK(hipEventRecord(h->step_ev[2], s)); }
    }
    phases &= ~(PH_MODEL | PH_LOGIC);
  }
  if (phases & PH_MODEL) {
    if (timed) HIPCHK(hipEventRecord(h->step_ev[0], s));
    hipLaunchKernelGGL(model_kernel, dim3(nb), dim3(SBLOCK), MODEL_CT_LDS_BYTES, s, P, actions, discrete,
                       terminal_obs != nullptr, policy, seed, step, obs_in);
    HIPCHK(hipGetLastError());
    if (h->car_contact) {
      hipLaunchKernelGGL(car_contact_kernel, dim3(nb), dim3(SBLOCK), CC_LDS_BYTES, s, P);
      HIPCHK(hipGetLastError());
    }
    if (timed) HIPCHK(hipEventRecord(h->step_ev[1], s));
  }
  if (phases & PH_LOGIC) {
    hipLaunchKernelGGL(logic_kernel, dim3(nb), dim3(SBLOCK), 0, s, P, obs, reward, car_flags,
                       env_flags, auto_reset, terminal_obs);
    HIPCHK(hipGetLastError());
    if (timed) HIPCHK(hipEventRecord(h->step_ev[2], s));
  }
  if (phases & PH_SENSOR) {
    launch_sensors_impl(h, P, nb, obs, terminal_obs, auto_reset ? 3 : 1, s, sensor_impl());
    HIPCHK(hipGetLastError());
    if (timed) HIPCHK(hipEventRecord(h->step_ev[3], s));
  }
  return 0;
}

extern "C" int nascar_set_step_events(NascarHandle* h, void* const* events, int32_t n) {
  if (!h) return fail("null argument");
  if (n == 0) { for (auto& e : h->step_ev) e = nullptr; return 0; }
  if (n != 4 || !events) return fail("step events: pass 4 events (or 0 to switch them off), got %d", n);
  for (int k = 0; k < 4; ++k) {
    if (!events[k]) return fail("step event %d is null", k);
    h->step_ev[k] = (hipEvent_t)events[k];
  }
  return 0;
}

static int step_impl(NascarHandle* h, const void* actions, int32_t discrete, int policy, uint64_t seed, int64_t step,
                     float* obs, float* reward, uint8_t* car_flags, uint8_t* env_flags, int32_t auto_reset,
                     float* terminal_obs, void* stream) {
  h->pristine = false;
  if (prepare(h, (hipStream_t)stream)) return -1;
  Params P = make_params(h);
  // Whole grid on the caller's stream: splitting one step over streams needs a fork and a join per step, and
  // the per-step barrier measured slower than one grid (tools/streams_exp.py: 2 / 4 shards 0.252 / 0.277 ms vs
  // 0.224 ms).  Shards pay off only when they run many steps unsynchronised: the sharded nascar_rollout.
  const bool rt = h->rt_on && auto_reset;
  uint8_t* ef = (rt && !env_flags) ? h->d_rt_flags : env_flags;
  if (launch_step_range(h, P, h->nblocks, actions, discrete, policy, seed, step, obs, obs, reward, car_flags, ef, auto_reset,
                        terminal_obs, (hipStream_t)stream))
    return -1;
  return rt ? rt_after_step(h, P, ef, obs, (hipStream_t)stream) : 0;
}

// Sharded rollout: the workgroups split into S contiguous ranges (shards of whole envs), each stepped `steps`
// times by per-step launches on its own stream -- shard 0 on the caller's stream, shards 1.. on internal streams
// forked from it at the start and joined into it at the end (S streams in all: the process has few hardware
// queues, GPU_MAX_HW_QUEUES = 4, and two shards on one queue run one after the other).  Envs are independent, so
// a shard needs only its own previous step: while one shard's slowest cars finish a step (the Box2D TOI chains
// that set each kernel's tail) the other shards' kernels fill the idle CUs, and the shards drift apart by up to
// the whole rollout.  Same kernels and arguments as nascar_step_driven, so the results equal `steps` x
// nascar_step_driven bit for bit (tests/test_gpu_rollout.py).
// Policy 2 (the SAC actor): each shard runs the actor on its own cars' observations, then steps them -- the
// cars of a shard are contiguous when the block map is the identity (one track, envs in workgroup order);
// otherwise the rollout runs as one shard.
static void launch_actor(NascarHandle* h, int n, const float* obs, float* actions, void* stream);
static int rollout_sharded(NascarHandle* h, int S, int32_t policy, uint64_t seed, int64_t step0, int32_t steps, float* obs,
                           float* reward, uint8_t* car_flags, uint8_t* env_flags, int32_t auto_reset, int32_t traj,
                           hipStream_t stream) {
  S = std::max(1, std::min(S, h->nblocks));
  const bool rt = h->rt_on && auto_reset;
  if (h->rt_on) S = 1;   // random-track mode: the block map changes between steps, so no shard owns a fixed set of envs
  const bool actor = policy == 2;
  if (actor) {
    if (!h->d_actor) return fail("policy 2 needs an actor (nascar_set_actor)");
    if ((uintptr_t)obs & 7) return fail("actor obs must be 8-byte aligned");
    if (!h->map_identity) S = 1;
    if (!h->d_ro_act) HIPCHK(hipMalloc(&h->d_ro_act, sizeof(float) * 2 * (size_t)h->N));
  }
  if ((int)h->sub_stream.size() < S - 1 || (S > 1 && !h->ev_fork)) {   // on the handle's device, whatever is current
    int cur = 0;
    HIPCHK(hipGetDevice(&cur));
    if (cur != h->cfg.device) HIPCHK(hipSetDevice(h->cfg.device));
    bool ok = true;
    while (ok && (int)h->sub_stream.size() < S - 1) {   // a stream and its join event, both or neither
      hipStream_t st; hipEvent_t ev;
      ok = hipStreamCreateWithFlags(&st, hipStreamNonBlocking) == hipSuccess;
      if (ok && hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) { hipStreamDestroy(st); ok = false; }
      if (ok) { h->sub_stream.push_back(st); h->ev_join.push_back(ev); }
    }
    if (ok && !h->ev_fork) ok = hipEventCreateWithFlags(&h->ev_fork, hipEventDisableTiming) == hipSuccess;
    if (cur != h->cfg.device) hipSetDevice(cur);
    if (!ok) return fail("creating the rollout shard streams failed");
  }
  auto shard_stream = [&](int s) { return s == 0 ? stream : h->sub_stream[s - 1]; };
  const Params P0 = make_params(h);
  if (S > 1) {
    HIPCHK(hipEventRecord(h->ev_fork, stream));
    for (int s = 1; s < S; ++s) HIPCHK(hipStreamWaitEvent(shard_stream(s), h->ev_fork, 0));
  }
  const size_t NC = (size_t)h->N, E = (size_t)h->E;
  const bool obs_traj = (traj & NASCAR_TRAJ_OBS) != 0;   // obs = [steps + 1][N][38]: record 0 in, record k + 1 out
  auto enqueue = [&]() -> int {
    for (int k = 0; k < steps; ++k) {
      const size_t ko = traj ? (size_t)k : 0;
      float* o_in = obs_traj ? obs + (size_t)k * NC * 38 : obs;
      float* o_out = obs_traj ? obs + (size_t)(k + 1) * NC * 38 : obs;
      // phase-major enqueue (every shard's model launch, then every shard's logic, then sensors): each stream's
      // order is unchanged, but a shard's first launch of the call is queued ~6 us (one launch) after the previous
      // shard's instead of ~18 us (three), so the shards start together
      for (int ph = 0; ph < 3; ++ph) {
        for (int s = 0; s < S; ++s) {
          const int b0 = (int)((int64_t)h->nblocks * s / S), b1 = (int)((int64_t)h->nblocks * (s + 1) / S);
          Params P = P0;
          P.blk0 = b0;
          if (actor && ph == 0) {
            const size_t c0 = S == 1 ? 0 : (size_t)b0 * h->epb * h->C;
            const size_t c1 = S == 1 ? NC : std::min((size_t)b1 * h->epb, E) * h->C;
            if (c1 > c0) launch_actor(h, (int)(c1 - c0), o_in + c0 * 38, h->d_ro_act + c0 * 2, shard_stream(s));
            HIPCHK(hipGetLastError());
          }
          if (launch_step_range(h, P, b1 - b0, actor ? h->d_ro_act : nullptr, 0, actor ? -1 : policy, seed, step0 + k,
                                o_in, o_out, reward + ko * NC,
                                car_flags ? car_flags + ko * NC : nullptr,
                                env_flags ? env_flags + ko * E : (rt ? h->d_rt_flags : nullptr),
                                auto_reset, nullptr, shard_stream(s), 1 << ph, ph == 1))
            return -1;
        }
      }
      if (rt && rt_after_step(h, P0, env_flags ? env_flags + ko * E : h->d_rt_flags, o_out, stream)) return -1;
    }
    return 0;
  };
  const int rc = enqueue();
  // join every shard into the caller's stream even when a launch failed part way: the shard work already queued
  // must stay ordered before whatever the caller enqueues next (a reset, set_state, a reused tensor)
  int jrc = 0;
  for (int s = 1; s < S; ++s) {
    const hipError_t e1 = hipEventRecord(h->ev_join[s - 1], shard_stream(s));
    const hipError_t e2 = e1 == hipSuccess ? hipStreamWaitEvent(stream, h->ev_join[s - 1], 0) : e1;
    if (e2 != hipSuccess && !jrc && !rc) jrc = fail("joining rollout shard %d failed: %s", s, hipGetErrorString(e2));
  }
  return rc ? rc : jrc;
}

// Pipelined rollout (see pipe_step_kernel): the step kernel on the caller's stream, the sensor kernel on the first
// shard stream, both launched after the per-call counter reset and joined into the caller's stream at the end.  Calls
// are cut into chunks of at most PIPE_CHUNK steps (the ring holds one chunk's items).
#define PIPE_CHUNK 64
static int rollout_pipe(NascarHandle* h, int policy, uint64_t seed, int64_t step0, int steps, float* obs, float* reward,
                        uint8_t* car_flags, uint8_t* env_flags, int auto_reset, int traj, hipStream_t stream) {
  const int nb = h->nblocks, sub = (h->epb * h->C + PIPE_CARS - 1) / PIPE_CARS;
  if (sub > 32) return fail("pipelined rollout: at most %d cars per step workgroup", 32 * PIPE_CARS);
  const size_t per_step = (size_t)nb * sub, chunk = std::min<size_t>(PIPE_CHUNK, std::max<size_t>(1, 0x7FFFFFFFu / per_step));
  const size_t cap = per_step * std::min<size_t>(chunk, (size_t)steps);   // slots per XCD: a chunk's items
  if (h->pipe_cap < cap) {
    hipFree(h->d_pipe_ring); h->d_pipe_ring = nullptr; h->pipe_cap = 0;
    HIPCHK(hipMalloc(&h->d_pipe_ring, sizeof(unsigned long long) * 8 * cap));
    HIPCHK(hipMemsetAsync(h->d_pipe_ring, 0, sizeof(unsigned long long) * 8 * cap, stream));   // tag 0 is never a call's
    h->pipe_cap = cap;
  }
  if (!h->d_pipe_ctr) {
    HIPCHK(hipMalloc(&h->d_pipe_ctr, 320 * sizeof(unsigned)));
    HIPCHK(hipMemsetAsync(h->d_pipe_ctr, 0, 320 * sizeof(unsigned), stream));
  }
  if (h->pipe_nb < (size_t)nb) {
    hipFree(h->d_pipe_sdone); h->d_pipe_sdone = nullptr; h->pipe_nb = 0;
    HIPCHK(hipMalloc(&h->d_pipe_sdone, sizeof(unsigned) * nb));
    h->pipe_nb = nb;
  }
  if (h->sub_stream.empty() || !h->ev_fork) {   // one extra stream (the first shard stream) and its join event
    int cur = 0;
    HIPCHK(hipGetDevice(&cur));
    if (cur != h->cfg.device) HIPCHK(hipSetDevice(h->cfg.device));
    bool ok = true;
    if (h->sub_stream.empty()) {
      hipStream_t st; hipEvent_t ev;
      ok = hipStreamCreateWithFlags(&st, hipStreamNonBlocking) == hipSuccess;
      if (ok && hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) { hipStreamDestroy(st); ok = false; }
      if (ok) { h->sub_stream.push_back(st); h->ev_join.push_back(ev); }
    }
    if (ok && !h->ev_fork) ok = hipEventCreateWithFlags(&h->ev_fork, hipEventDisableTiming) == hipSuccess;
    if (cur != h->cfg.device) hipSetDevice(cur);
    if (!ok) return fail("creating the pipelined rollout's sensor stream failed");
  }
  const Params P = make_params(h);
  if (!h->d_params) {
    HIPCHK(hipMalloc(&h->d_params, sizeof(Params)));
    memset(&h->params_up, 0, sizeof(Params));
  }
  if (!h->params_valid || memcmp(&h->params_up, &P, sizeof(Params)) != 0) {   // stream-ordered upload when changed
    h->params_up = P; h->params_valid = true;
    HIPCHK(hipMemcpyAsync(h->d_params, &h->params_up, sizeof(Params), hipMemcpyHostToDevice, stream));
  }
  hipStream_t ss = h->sub_stream[0];
  const size_t NC = (size_t)h->N, E = (size_t)h->E;
  for (int k0 = 0; k0 < steps; k0 += (int)chunk) {
    const int kc = (int)std::min<size_t>(chunk, (size_t)(steps - k0));
    HIPCHK(hipMemsetAsync(h->d_pipe_ctr, 0, (PIPE_REG + 1) * sizeof(unsigned), stream));   // the per-call counters (not the error)
    HIPCHK(hipMemsetAsync(h->d_pipe_sdone, 0, sizeof(unsigned) * nb, stream));
    if (++h->pipe_seq == 0) h->pipe_seq = 1;
#ifdef NASCAR_AB_KNOBS   // diagnostic builds (tools/mklib.sh): printf milestones, variants, a shorter bound
    static const int dbg = getenv("NASCAR_PIPE_DEBUG") ? atoi(getenv("NASCAR_PIPE_DEBUG")) : 0;
    static const unsigned long long tmo = 100000ull * (unsigned long long)(getenv("NASCAR_PIPE_TIMEOUT_MS") ? atoi(getenv("NASCAR_PIPE_TIMEOUT_MS")) : 2000);
#else
    const int dbg = 0;
    const unsigned long long tmo = 100000ull * 2000;   // 2 s without progress fails the call
#endif
    PipeDev Q{h->d_pipe_ring, h->d_pipe_ctr, h->d_pipe_sdone, h->pipe_seq, (unsigned)h->pipe_cap, sub, nb, dbg, tmo};
    // the sensor stream starts after the resets, not after the step kernel (which waits on it)
    HIPCHK(hipEventRecord(h->ev_fork, stream));
    HIPCHK(hipStreamWaitEvent(ss, h->ev_fork, 0));
    const size_t ko = traj ? (size_t)k0 : 0;
    hipLaunchKernelGGL(pipe_step_kernel, dim3(nb), dim3(SBLOCK), MODEL_LOGIC_LDS_BYTES, stream, (const Params*)h->d_params, Q,
                       kc, policy, seed,
                       step0 + k0, obs, reward + ko * NC, car_flags ? car_flags + ko * NC : nullptr,
                       env_flags ? env_flags + ko * E : nullptr, auto_reset, traj);
    HIPCHK(hipGetLastError());
    hipLaunchKernelGGL(pipe_sensor_kernel, dim3(h->ro_pipe), dim3(64), 0, ss, (const Params*)h->d_params, Q, obs,
                       auto_reset ? 3 : 1);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(h->ev_join[0], ss));
    HIPCHK(hipStreamWaitEvent(stream, h->ev_join[0], 0));
  }
  return 0;
}
extern "C" int nascar_set_rollout_pipe(NascarHandle* h, int32_t sensor_workgroups) {
  if (!h) return fail("null argument");
  if (sensor_workgroups < 0 || sensor_workgroups > 65536) return fail("sensor workgroups must be in [0, 65536] (got %d)", sensor_workgroups);
  h->ro_pipe = sensor_workgroups;
  return 0;
}
extern "C" int nascar_rollout_pipe_status(NascarHandle* h, void* stream) {
  if (!h) return fail("null argument");
  if (!h->d_pipe_ctr) return 0;
  unsigned err = 0;
  HIPCHK(hipStreamSynchronize((hipStream_t)stream));
  HIPCHK(hipMemcpy(&err, h->d_pipe_ctr + PIPE_ERR, sizeof(unsigned), hipMemcpyDeviceToHost));
  if (err) HIPCHK(hipMemset(h->d_pipe_ctr + PIPE_ERR, 0, sizeof(unsigned)));
  return err ? 1 : 0;
}
extern "C" int nascar_get_rollout_streams(NascarHandle* h) { return h ? h->ro_streams : -1; }
extern "C" int nascar_set_rollout_streams(NascarHandle* h, int32_t streams) {
  if (!h) return fail("null argument");
  if (streams < 0 || streams > 16) return fail("rollout streams must be in [0, 16] (got %d)", streams);
  h->ro_streams = streams;
  return 0;
}

extern "C" int nascar_rollout(NascarHandle* h, int32_t policy, uint64_t seed, int64_t step0, int32_t steps, float* obs,
                              float* reward, uint8_t* car_flags, uint8_t* env_flags, int32_t auto_reset, int32_t traj,
                              void* stream) {
  if (!h || !obs || !reward) return fail("null argument");
  if (policy < 0 || policy > 3) return fail("rollout policy must be 0, 1, 2 or 3 (got %d)", policy);
  if (policy == 2 && h->ro_streams == 0) return fail("the fused rollout kernel has no actor (policy 2): use the sharded rollout");
  if (h->rt_on && h->ro_streams == 0)
    return fail("random-track mode needs the sharded rollout (rollout streams >= 1): the fused kernel keeps one block map");
  if (traj & ~(NASCAR_TRAJ_RECORDS | NASCAR_TRAJ_OBS)) return fail("unknown trajectory flags 0x%x", traj);
  if ((traj & NASCAR_TRAJ_OBS) && !(traj & NASCAR_TRAJ_RECORDS)) return fail("an obs trajectory needs the per-step records (traj bit 0)");
  if ((traj & NASCAR_TRAJ_OBS) && h->ro_streams == 0) return fail("obs trajectories need the sharded rollout (rollout streams >= 1)");
  if (steps < 0) return fail("steps must be >= 0");
  if (steps == 0) return 0;
  h->pristine = false;
  if (prepare(h, (hipStream_t)stream)) return -1;
  if (h->ro_pipe > 0 && policy != 2 && !h->rt_on && !h->car_contact && !(traj & NASCAR_TRAJ_OBS))
    return rollout_pipe(h, policy, seed, step0, steps, obs, reward, car_flags, env_flags, auto_reset, traj,
                        (hipStream_t)stream);
  if (h->ro_streams > 0)
    return rollout_sharded(h, h->ro_streams, policy, seed, step0, steps, obs, reward, car_flags, env_flags, auto_reset,
                           traj, (hipStream_t)stream);
  Params P = make_params(h);   // ro_streams == 0: the fused rollout_kernel
  if (!h->d_params) {
    HIPCHK(hipMalloc(&h->d_params, sizeof(Params)));
    memset(&h->params_up, 0, sizeof(Params));
  }
  if (!h->params_valid || memcmp(&h->params_up, &P, sizeof(Params)) != 0) {   // stream-ordered upload when changed
    h->params_up = P; h->params_valid = true;
    HIPCHK(hipMemcpyAsync(h->d_params, &h->params_up, sizeof(Params), hipMemcpyHostToDevice, (hipStream_t)stream));
  }
  // >= 2 float4 per wall of the largest track; the car-car extension's scratch after it
  const size_t lds = ((h->max_sensor_lds + 15) & ~(size_t)15) + (h->car_contact ? CC_LDS_BYTES : 0);
  hipLaunchKernelGGL(rollout_kernel, dim3(h->nblocks), dim3(SBLOCK), lds, (hipStream_t)stream, (const Params*)h->d_params,
                     steps, policy, seed, step0, obs, reward, car_flags, env_flags, auto_reset, traj);
  HIPCHK(hipGetLastError());
  return 0;
}

extern "C" int nascar_get_info(NascarHandle* h, double* info, void* stream) {
  if (!h || !info) return fail("null argument");
  if (prepare(h, (hipStream_t)stream)) return -1;
  Params P = make_params(h);
  hipLaunchKernelGGL(info_kernel, dim3(h->nblocks), dim3(SBLOCK), 0, (hipStream_t)stream, P, info);
  HIPCHK(hipGetLastError());
  return 0;
}

// ------------------------------------------------------------------ random-track mode (host side)
extern "C" int nascar_track_draw(int32_t n, const uint64_t* seeds, const int32_t* k, const int32_t* current,
                                 const int32_t* tracks, int32_t ntracks, int32_t* out) {
  if (n < 0 || (n > 0 && (!seeds || !k || !current || !out)) || (ntracks > 0 && !tracks)) return fail("bad argument");
  for (int32_t i = 0; i < n; ++i) out[i] = rt_draw(seeds[i], k[i], current[i], tracks, ntracks);
  return 0;
}
extern "C" int nascar_set_random_tracks(NascarHandle* h, const int32_t* tracks, int32_t ntracks, const uint64_t* seeds,
                                        const int32_t* draws, void* stream) {
  if (!h) return fail("null argument");
  const hipStream_t s = (hipStream_t)stream;
  const size_t E = (size_t)h->E;
  if (ntracks == 0) {   // off: the device's assignment becomes the host's, the host builds the block map again
    if (h->rt_on) {
      std::vector<int> et(E);
      HIPCHK(hipMemcpyAsync(et.data(), h->d_rt_env_track, sizeof(int) * E, hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
      h->env_track = et;
      h->rt_on = 0; h->rt_ntracks = 0; h->dirty_tracks = true;
    }
    return 0;
  }
  if (!tracks || !seeds) return fail("null argument");
  if (ntracks < 0 || ntracks > RT_MAX_TRACKS) return fail("random tracks: %d ids (at most %d)", ntracks, RT_MAX_TRACKS);
  if ((int)h->tracks.size() > RT_MAX_TRACKS) return fail("random-track mode supports at most %d loaded tracks", RT_MAX_TRACKS);
  for (int i = 0; i < ntracks; ++i) {
    if (tracks[i] < 0 || tracks[i] >= (int)h->tracks.size()) return fail("random tracks: bad track id %d", tracks[i]);
    for (int j = 0; j < i; ++j) if (tracks[j] == tracks[i]) return fail("random tracks: track id %d listed twice", tracks[i]);
  }
  if (draws) for (size_t e = 0; e < E; ++e) if (draws[e] < 0) return fail("env %zu: negative draw count", e);
  if (!h->pending_track.empty()) {
    for (size_t e = 0; e < E; ++e)
      if (h->pending_track[e] != h->env_track[e])
        return fail("env %zu has a track change pending (nascar_set_env_tracks): reset it before random-track mode", e);
    h->pending_track.clear();
  }
  if (!h->d_rt) {
    const size_t o_dr = align256(sizeof(int) * E), o_sd = o_dr + align256(sizeof(int) * E),
                 o_tr = o_sd + align256(sizeof(uint64_t) * E), o_dy = o_tr + align256(sizeof(int) * RT_MAX_TRACKS),
                 o_fl = o_dy + 256, total = o_fl + align256(E);
    HIPCHK(hipMalloc(&h->d_rt, total));
    HIPCHK(hipMemsetAsync(h->d_rt, 0, total, s));
    char* b = (char*)h->d_rt;
    h->d_rt_env_track = (int*)b; h->d_rt_draws = (int*)(b + o_dr); h->d_rt_seed = (uint64_t*)(b + o_sd);
    h->d_rt_tracks = (int*)(b + o_tr); h->d_rt_dirty = (int*)(b + o_dy); h->d_rt_flags = (uint8_t*)(b + o_fl);
  }
  std::vector<int> dr(E, 0);
  if (draws) for (size_t e = 0; e < E; ++e) dr[e] = draws[e];
  if (!h->rt_on) HIPCHK(hipMemcpyAsync(h->d_rt_env_track, h->env_track.data(), sizeof(int) * E, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(h->d_rt_draws, dr.data(), sizeof(int) * E, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(h->d_rt_seed, seeds, sizeof(uint64_t) * E, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(h->d_rt_tracks, tracks, sizeof(int) * ntracks, hipMemcpyHostToDevice, s));
  HIPCHK(hipStreamSynchronize(s));   // (pageable, caller-owned host arrays)
  h->rt_on = 1; h->rt_ntracks = ntracks; h->dirty_tracks = true;
  return 0;
}
extern "C" int nascar_get_env_tracks(NascarHandle* h, int32_t* env_track, int32_t* draws, void* stream) {
  if (!h) return fail("null argument");
  const hipStream_t s = (hipStream_t)stream;
  const size_t bytes = sizeof(int) * (size_t)h->E;
  if (h->rt_on) {
    if (env_track) HIPCHK(hipMemcpyAsync(env_track, h->d_rt_env_track, bytes, hipMemcpyDeviceToDevice, s));
    if (draws) HIPCHK(hipMemcpyAsync(draws, h->d_rt_draws, bytes, hipMemcpyDeviceToDevice, s));
    return 0;
  }
  if (env_track) {
    HIPCHK(hipMemcpyAsync(env_track, h->env_track.data(), bytes, hipMemcpyHostToDevice, s));
    HIPCHK(hipStreamSynchronize(s));
  }
  if (draws) HIPCHK(hipMemsetAsync(draws, 0, bytes, s));
  return 0;
}
extern "C" int nascar_vec_post(NascarHandle* h, const float* reward, const uint8_t* env_flags, double* ep_ret,
                               int64_t* ep_len, uint8_t* done, double* snap_ret, int64_t* snap_len, void* stream) {
  if (!h || !reward || !env_flags || !ep_ret || !ep_len || !done || !snap_ret || !snap_len) return fail("null argument");
  hipLaunchKernelGGL(vec_post_kernel, dim3((h->E + 255) / 256), dim3(256), 0, (hipStream_t)stream, h->E, h->C, reward,
                     env_flags, ep_ret, ep_len, done, snap_ret, snap_len);
  HIPCHK(hipGetLastError());
  return 0;
}
extern "C" int nascar_check_actions(NascarHandle* h, const void* actions, int32_t discrete, int32_t* bad, void* stream) {
  if (!h || !actions || !bad) return fail("null argument");
  const int n = h->N * (discrete ? 1 : 2);
  hipLaunchKernelGGL(action_check_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, n, actions,
                     (int)(discrete != 0), bad);
  HIPCHK(hipGetLastError());
  return 0;
}

extern "C" int nascar_set_car_contact(NascarHandle* h, int32_t enable) {
  if (!h) return fail("null argument");
  h->car_contact = enable ? 1 : 0;
  return 0;
}

extern "C" int nascar_set_perf_history(NascarHandle* h, int32_t enable, void* stream) {
  if (!h) return fail("null argument");
  if (!enable) { if (h->d_vhist) { HIPCHK(hipStreamSynchronize((hipStream_t)stream)); hipFree(h->d_vhist); h->d_vhist = nullptr; } return 0; }
  if (h->d_vhist) return 0;
  const size_t bytes = sizeof(float) * (size_t)VH_RING * h->N;
  HIPCHK(hipMalloc(&h->d_vhist, bytes));
  // every slot NaN: until an episode has written the whole window since the enable, info reports perf_count -1
  // (enabling mid-episode would otherwise count the steps taken before it as zero speeds)
  HIPCHK(hipMemsetAsync(h->d_vhist, 0xFF, bytes, (hipStream_t)stream));
  return 0;
}

extern "C" int64_t nascar_state_bytes(NascarHandle* h) { return h ? (int64_t)h->arena_bytes : -1; }
extern "C" int nascar_get_state(NascarHandle* h, void* dst, void* stream) {
  if (!h || !dst) return fail("null argument");
  HIPCHK(hipMemcpyAsync(dst, h->arena, h->arena_bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return 0;
}
extern "C" int nascar_set_state(NascarHandle* h, const void* src, void* stream) {
  if (!h || !src) return fail("null argument");
  h->pristine = false;
  HIPCHK(hipMemcpyAsync(h->arena, src, h->arena_bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return 0;
}

static void launch_actor(NascarHandle* h, int n, const float* obs, float* actions, void* stream);
extern "C" int nascar_policy_actions(NascarHandle* h, int32_t policy, uint64_t seed, int64_t step, const float* obs,
                                     float* actions, void* stream) {
  if (!h || !actions) return fail("null argument");
  if (policy < 0 || policy > 3) return fail("unknown policy %d", policy);
  if (policy >= 1 && !obs) return fail("policy %d needs obs", policy);
  if (policy == 2) {
    if (!h->d_actor) return fail("policy 2 needs an actor (nascar_set_actor)");
    if (((uintptr_t)obs | (uintptr_t)actions) & 7) return fail("actor obs/actions must be 8-byte aligned");
    launch_actor(h, h->N, obs, actions, stream);
    HIPCHK(hipGetLastError());
    return 0;
  }
  int nb = (h->N + 255) / 256;
  hipLaunchKernelGGL(policy_kernel, dim3(nb), dim3(256), 0, (hipStream_t)stream, h->N, policy, seed, step, obs, actions, h->d_ctl);
  HIPCHK(hipGetLastError());
  return 0;
}

// ------------------------------------------------------------------ test hook: b2Rot::Set numerics
__global__ void sincos_kernel(const float* x, float* s, float* c, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) glibc_sincosf(x[i], &s[i], &c[i]);
}
static uint16_t f32_to_bf16_rne(float f) {
  uint32_t u; memcpy(&u, &f, 4);
  if ((u & 0x7F800000u) == 0x7F800000u && (u & 0x007FFFFFu)) return (uint16_t)((u >> 16) | 0x40);   // quiet NaN
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

// SB3 SAC MlpPolicy actor (game/control/sac_control_class.py:80-115), PyTorch layouts:
// w1 [256][38], b1 [256], w2 [256][256], b2 [256], w3 (mu) [2][256], b3 [2]; host float32.
extern "C" int nascar_set_actor(NascarHandle* h, const float* w1, const float* b1, const float* w2, const float* b2,
                                const float* w3, const float* b3, int32_t obs_dim, int32_t hidden, int32_t act_dim) {
  if (!h || !w1 || !b1 || !w2 || !b2 || !w3 || !b3) return fail("null argument");
  if (obs_dim != ACT_OBS || hidden != ACT_H || act_dim != ACT_OUT)
    return fail("actor shape %dx%dx%d unsupported (need 38x256x2: SB3 MlpPolicy net_arch [256, 256])", obs_dim, hidden, act_dim);
  std::vector<uint16_t> w1p((size_t)ACT_H * ACT_K, 0), w2p((size_t)ACT_H * ACT_H);
  for (int o = 0; o < ACT_H; ++o) {
    for (int i = 0; i < ACT_OBS; ++i) w1p[(size_t)o * ACT_K + i] = f32_to_bf16_rne(w1[(size_t)o * ACT_OBS + i]);
    // b1 rides in the two extra K columns (the observation tile holds 1.0 there): hi + lo bf16 halves
    const uint16_t hi = f32_to_bf16_rne(b1[o]);
    const uint32_t hb = (uint32_t)hi << 16;
    float hf; memcpy(&hf, &hb, 4);
    w1p[(size_t)o * ACT_K + ACT_OBS] = hi;
    w1p[(size_t)o * ACT_K + ACT_OBS + 1] = f32_to_bf16_rne(b1[o] - hf);
  }
  // layer-2 A fragments in the k order of the layer-1 accumulator registers (nascar_actor.h)
  for (int o = 0; o < 8; ++o)
    for (int q = 0; q < 8; ++q)
      for (int s = 0; s < 2; ++s)
        for (int r = 0; r < 32; ++r)
          for (int hh = 0; hh < 2; ++hh)
            for (int j = 0; j < 8; ++j) {
              const int row = 32 * o + r, col = 32 * q + 16 * s + 8 * (j >> 2) + 4 * hh + (j & 3);
              w2p[((((size_t)(o * 8 + q) * 2 + s) * 2 + hh) * 32 + r) * 8 + j] = f32_to_bf16_rne(w2[(size_t)row * ACT_H + col]);
            }
  // layer-3 A fragments: W3' rows 0-3 = hi(w3[0]), hi(w3[1]), lo(w3[0]), lo(w3[1]) in the k order of the
  // layer-2 accumulator registers (rows 4-31 are zero and not stored)
  std::vector<uint16_t> w3p((size_t)8 * 2 * 2 * 4 * 8);
  for (int o = 0; o < 8; ++o)
    for (int s = 0; s < 2; ++s)
      for (int hh = 0; hh < 2; ++hh)
        for (int r = 0; r < 4; ++r)
          for (int j = 0; j < 8; ++j) {
            const int col = 32 * o + 16 * s + 8 * (j >> 2) + 4 * hh + (j & 3);
            const float w = w3[(size_t)(r & 1) * ACT_H + col];
            const uint16_t hi = f32_to_bf16_rne(w);
            const uint32_t hb = (uint32_t)hi << 16;
            float hf; memcpy(&hf, &hb, 4);
            w3p[((((size_t)o * 2 + s) * 2 + hh) * 4 + r) * 8 + j] = r < 2 ? hi : f32_to_bf16_rne(w - hf);
          }
  const size_t o_w1 = 0, o_w2 = o_w1 + w1p.size() * 2, o_b2 = o_w2 + w2p.size() * 2,
               o_w3 = o_b2 + ACT_H * 4, o_b3 = o_w3 + w3p.size() * 2, total = o_b3 + 64;
  if (!h->d_actor) HIPCHK(hipMalloc(&h->d_actor, total));
  char* d = (char*)h->d_actor;
  HIPCHK(hipMemcpy(d + o_w1, w1p.data(), w1p.size() * 2, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(d + o_w2, w2p.data(), w2p.size() * 2, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(d + o_b2, b2, ACT_H * 4, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(d + o_w3, w3p.data(), w3p.size() * 2, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(d + o_b3, b3, ACT_OUT * 4, hipMemcpyHostToDevice));
  h->actor.w1p = (const bf16x8*)(d + o_w1); h->actor.w2p = (const bf16x8*)(d + o_w2);
  h->actor.b2 = (const float*)(d + o_b2); h->actor.w3p = (const bf16x8*)(d + o_w3); h->actor.b3 = (const float*)(d + o_b3);
  {   // float32 copies for the reference-precision kernel: W1 and W2 transposed ([k][unit])
    std::vector<float> f((size_t)ACT_OBS * ACT_H + ACT_H + (size_t)ACT_H * ACT_H + ACT_H + 2 * ACT_H + 2);
    float* p = f.data();
    float* w1t = p; p += (size_t)ACT_OBS * ACT_H;
    float* b1c = p; p += ACT_H;
    float* w2t = p; p += (size_t)ACT_H * ACT_H;
    float* b2c = p; p += ACT_H;
    float* w3c = p; p += 2 * ACT_H;
    float* b3c = p;
    for (int o = 0; o < ACT_H; ++o)
      for (int i = 0; i < ACT_OBS; ++i) w1t[(size_t)i * ACT_H + o] = w1[(size_t)o * ACT_OBS + i];
    for (int o = 0; o < ACT_H; ++o)
      for (int i = 0; i < ACT_H; ++i) w2t[(size_t)i * ACT_H + o] = w2[(size_t)o * ACT_H + i];
    memcpy(b1c, b1, 4 * ACT_H); memcpy(b2c, b2, 4 * ACT_H); memcpy(w3c, w3, 8 * ACT_H); memcpy(b3c, b3, 8);
    if (!h->d_actor32) HIPCHK(hipMalloc(&h->d_actor32, f.size() * 4));
    HIPCHK(hipMemcpy(h->d_actor32, f.data(), f.size() * 4, hipMemcpyHostToDevice));
    const float* d32 = (const float*)h->d_actor32;
    h->actor32.w1t = d32 + (w1t - f.data()); h->actor32.b1 = d32 + (b1c - f.data());
    h->actor32.w2t = d32 + (w2t - f.data()); h->actor32.b2 = d32 + (b2c - f.data());
    h->actor32.w3 = d32 + (w3c - f.data()); h->actor32.b3 = d32 + (b3c - f.data());
  }
  return 0;
}

extern "C" int nascar_set_actor_precision(NascarHandle* h, int32_t fp32) {
  if (!h) return fail("null argument");
  if (fp32 != 0 && fp32 != 1) return fail("precision must be 0 (bf16 MFMA) or 1 (fp32)");
  h->actor_fp32 = fp32;
  return 0;
}

static void launch_actor(NascarHandle* h, int n, const float* obs, float* actions, void* stream) {
#ifdef NASCAR_AB_KNOBS
  static const int fp32_valu = getenv("NASCAR_ACTOR_FP32_VALU") != nullptr;   // A/B tools builds: the f32 VALU kernel
#else
  const int fp32_valu = 0;
#endif
  if (h->actor_fp32 && !fp32_valu) {   // reference precision on the f32 MFMA: one wave per 32 observations
    const int tiles = (n + 31) / 32;
    hipLaunchKernelGGL(actor_mfma32_kernel, dim3((tiles + AM_WAVES - 1) / AM_WAVES), dim3(64 * AM_WAVES), 0,
                       (hipStream_t)stream, n, obs, actions, h->actor32);
  } else if (h->actor_fp32) {
    static int cus = 0;
    if (!cus) { int dev = 0; hipGetDevice(&dev); hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev); if (cus <= 0) cus = 256; }
    const int tiles = (n + AF_TILE - 1) / AF_TILE;
    hipLaunchKernelGGL(actor_fp32_kernel, dim3(std::max(1, std::min(tiles, 2 * cus))), dim3(256), 0, (hipStream_t)stream,
                       n, obs, actions, h->actor32);
  } else {
    hipLaunchKernelGGL(actor_kernel, dim3(actor_grid(n)), dim3(64 * ACT_WAVES), 0, (hipStream_t)stream, n, obs, actions, h->actor);
  }
}

// Actor forward on an arbitrary device batch: obs [n][38] float32 -> actions [n][2] float32.
extern "C" int nascar_actor_forward(NascarHandle* h, const float* obs, int32_t n, float* actions, void* stream) {
  if (!h || !obs || !actions || n < 0) return fail("bad argument");
  if (!h->d_actor) return fail("no actor loaded (nascar_set_actor)");
  if (((uintptr_t)obs | (uintptr_t)actions) & 7) return fail("actor obs/actions must be 8-byte aligned");
  if (n == 0) return 0;
  launch_actor(h, n, obs, actions, stream);
  HIPCHK(hipGetLastError());
  return 0;
}

extern "C" int nascar_debug_sincosf(const float* x, float* s, float* c, int32_t n, void* stream) {
  if (!x || !s || !c || n < 0) return fail("bad argument");
  hipLaunchKernelGGL(sincos_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, x, s, c, n);
  HIPCHK(hipGetLastError());
  return 0;
}

// Sensor test hook: car n's pose hand-off set to poses[n] = (x, y, angle) (float32, the body position and
// angle the sensors read), then one sensor launch: impl 1 = ray_sensor_kernel (beam lists), 0 = the
// wall-group sensor_kernel.  Writes obs[n * 38 + 22 .. 37]; other obs entries are left untouched.
__global__ void debug_pose_kernel(Params P, const float* poses) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= P.N) return;
  const float a = poses[3 * n + 2];
  P.pose[n] = make_float4(poses[3 * n], poses[3 * n + 1], a, __int_as_float(PM_A_OBS));
  double s0, c0;
  sincos((double)a, &s0, &c0);
  P.pose_cs[n] = make_double2(c0, s0);
}
extern "C" int nascar_debug_sensors(NascarHandle* h, const float* poses, float* obs, int32_t impl, void* stream) {
  if (!h || !poses || !obs) return fail("null argument");
  if (prepare(h, (hipStream_t)stream)) return -1;
  Params P = make_params(h);
  hipLaunchKernelGGL(debug_pose_kernel, dim3((h->N + 255) / 256), dim3(256), 0, (hipStream_t)stream, P, poses);
  HIPCHK(hipGetLastError());
  launch_sensors_impl(h, P, h->nblocks, obs, nullptr, 1, stream, impl);
  HIPCHK(hipGetLastError());
  return 0;
}

// Test hook: the current workgroup layout (block map) into caller device buffers -- blk_track [cap_blocks] and
// blk_env [cap_blocks * epb] int32 -- as the next launch would use it (prepare() first); returns the grid size
// (workgroups launched; in random-track mode the workgroups past the last track's are empty, track -1), or < 0.
extern "C" int nascar_debug_block_map(NascarHandle* h, int32_t* blk_track, int32_t* blk_env, int32_t cap_blocks,
                                      void* stream) {
  if (!h || !blk_track || !blk_env) return fail("null argument");
  if (prepare(h, (hipStream_t)stream)) return -1;
  if (cap_blocks < h->nblocks) return fail("block map needs %d workgroups, buffer holds %d", h->nblocks, cap_blocks);
  HIPCHK(hipMemcpyAsync(blk_track, h->d_blk_track, sizeof(int) * h->nblocks, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  HIPCHK(hipMemcpyAsync(blk_env, h->d_blk_env, sizeof(int) * (size_t)h->nblocks * h->epb, hipMemcpyDeviceToDevice,
                        (hipStream_t)stream));
  return h->nblocks;
}

#ifdef NASCAR_PROFILE
extern "C" int nascar_debug_profile(unsigned long long* dev_buf) {
  HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_prof), &dev_buf, sizeof(dev_buf)));
  return 0;
}
#endif
#ifdef NASCAR_DEBUG
extern "C" int nascar_debug_tap(double* dev_buf, int32_t car) {
  HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_dbg), &dev_buf, sizeof(dev_buf)));
  HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_dbg_car), &car, sizeof(car)));
  return 0;
}
#endif
