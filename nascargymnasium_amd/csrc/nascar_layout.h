// nascar_layout.h -- HBM layout of the batched CarEnv state (device + host).
//
// N = E*C cars, car index n = env * C + car.  Hot scalar state is SoA
// (field-major: value of field f for car n at base_f[n]) so a wavefront of 64
// cars reads each field with one coalesced 256-B (f32) / 512-B (f64) access.
// Variable-length per-car lists (Box2D contacts, listener collisions) are AoS per
// car, read only when the car has contacts.
#pragma once
#include <stdint.h>

namespace nascar {

#define MAXC 16          // Box2D contacts kept per car world (fat-AABB pairs); overflow -> error flag
#define MAX_ISLAND 8     // touching contacts solved per island (overflow -> error flag)

enum { CT_TOUCH = 1, CT_ENABLED = 2, CT_ISLAND = 4, CT_TOI = 8 };

struct DPoint { float lx, ly, ni, ti; uint32_t id; };
struct DContact {            // b2Contact + its b2Manifold (face manifolds only)
  int wall, flags, mtype, pointCount;
  float lnx, lny, lpx, lpy;  // localNormal, localPoint
  DPoint pt[2];
  float toi; int toiCount;
};

// float32 per-car fields
#define NASCAR_F32_FIELDS(X) \
  X(cx) X(cy) X(a) X(vx) X(vy) X(w) X(qs) X(qc) X(xpx) X(xpy) X(sleep) X(invdt0) \
  X(flox) X(floy) X(fhix) X(fhiy) X(cum_reward) X(cum_reward_info)
// float64 per-car fields (Python floats in the reference)
#define NASCAR_F64_FIELDS(X) \
  X(rpm) X(pvx) X(pvy) X(lfm) X(slip) X(bank) \
  X(load0) X(load1) X(load2) X(load3) X(temp0) X(temp1) X(temp2) X(temp3) \
  X(wear0) X(wear1) X(wear2) X(wear3) X(imp) \
  X(lt_start) X(lt_cur) X(lt_last) X(lt_best) X(lt_px) X(lt_py) X(lt_dist) \
  X(cum_impact) X(stuck_dur) X(stuck_sx) X(stuck_sy) X(prev_px) X(prev_py) \
  X(prog_hist) X(back) X(prev_back) X(imp_at_obs)
// int32 per-car fields
#define NASCAR_I32_FIELDS(X) \
  X(awake) X(nct) X(overflow) X(acc_len) X(acc_head) X(imp_present) X(nact) \
  X(lt_timing) X(lt_has_last) X(lt_has_best) X(lt_crossed) X(lt_has_pos) X(lt_laps) \
  X(disabled) X(has_stuck_start) X(first_step) X(prev_laps)

#define NASCAR_COUNT(f) +1
enum { N_F32 = 0 NASCAR_F32_FIELDS(NASCAR_COUNT), N_F64 = 0 NASCAR_F64_FIELDS(NASCAR_COUNT),
       N_I32 = 0 NASCAR_I32_FIELDS(NASCAR_COUNT) };
#define NASCAR_ENUM_F32(f) F32_##f,
#define NASCAR_ENUM_F64(f) F64_##f,
#define NASCAR_ENUM_I32(f) I32_##f,
enum { NASCAR_F32_FIELDS(NASCAR_ENUM_F32) F32_END };
enum { NASCAR_F64_FIELDS(NASCAR_ENUM_F64) F64_END };
enum { NASCAR_I32_FIELDS(NASCAR_ENUM_I32) I32_END };

// per-env state: sim_time (f64), created, pending, term_reason, terminated, truncated (i32)
enum { E_CREATED, E_PENDING, E_REASON, E_TERMINATED, E_TRUNCATED, N_EI32 };

// info vector per car written by nascar_get_info (float64)
enum {
  INFO_X, INFO_Y, INFO_VX, INFO_VY, INFO_ANGLE, INFO_OMEGA, INFO_SPEED, INFO_LAP_COUNT, INFO_LAST_LAP,
  INFO_BEST_LAP, INFO_IS_TIMING, INFO_CUR_LAP_TIME, INFO_LAP_DIST, INFO_HAS_CROSSED, INFO_DISABLED,
  INFO_CUM_REWARD, INFO_CUM_IMPACT, INFO_ON_TRACK, INFO_RPM, INFO_SIM_TIME, INFO_NCT, INFO_ERROR, INFO_PROGRESS,
  INFO_PERF_COUNT, INFO_PERF_MAX, INFO_PERF_FIRST, N_INFO
};

// Car.velocity_history (src/car.py:173, 384-386; deque(maxlen=VELOCITY_HISTORY_SIZE = 600)) for
// Car.validate_performance (src/car.py:1060-1098): per car, the body speed after each step, ring slot
// (steps since reset) % VH_RING, layout [VH_RING][N] float32 (b2Vec2::Length is float32).  Optional
// (nascar_set_perf_history); VH_RING > 600 so a step's write never lands in the window it is read with.
#define VH_SIZE 600
#define VH_RING 640

// car flag bits (nascar_step car_flags output)
enum { CF_DISABLED = 1, CF_JUST_DISABLED = 2, CF_COLLISION = 4, CF_LAP = 8, CF_ERROR = 128 };
// env flag bits (nascar_step env_flags output); bits 4..6 = termination reason code
enum { EF_TERMINATED = 1, EF_TRUNCATED = 2, EF_RESET = 8 };

}  // namespace nascar
