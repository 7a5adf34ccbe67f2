/*
 * include/nascar.h -- C ABI of the MI355X-native batched CarEnv (libnascar.so).
 *
 * Drop-in boundary for the reference's hot path: the Gymnasium CarEnv
 * step()/reset() of heihachi78/NascarGymnasium (src/car_env.py:678-803,
 * :316-535), whose per-car internals -- CarPhysics (src/car_physics.py),
 * Car/TyreManager/Tyre (src/car.py, src/tyre_manager.py, src/tyre.py),
 * DistanceSensor (src/distance_sensor.py), LapTimer (src/lap_timer.py) and the
 * Box2D calls they make through box2d-py SWIG -- run here as one fused HIP
 * kernel over E envs x C cars.  The Python CarEnv / batched VecEnv in
 * nascargymnasium_amd/ binds these entry points with ctypes.
 *
 * Conventions: every buffer argument of nascar_step/nascar_reset is a
 * caller-owned DEVICE pointer (e.g. torch tensor .data_ptr()); launches are
 * asynchronous on the caller's HIP stream (hipStream_t passed as void*).
 * Return code 0 = ok, negative = error; nascar_last_error() has the text.
 * No C++ exception crosses the ABI.  A handle is not thread-safe.
 */
#ifndef NASCAR_H
#define NASCAR_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct NascarHandle NascarHandle;

typedef struct NascarConfig {
    int32_t num_envs;        /* E */
    int32_t num_cars;        /* C in [1, 10] (src/constants/car_specs.py:50 MAX_CARS); up to 64 allowed */
    int32_t reset_on_lap;    /* CarEnv(reset_on_lap=...) (src/car_env.py:84) */
    int32_t device;          /* HIP device ordinal */
    double start_x, start_y, start_angle;   /* CarEnv start pose (src/car_env.py:114-115, 235-241) */
} NascarConfig;

/* CarEnv.__init__ (src/car_env.py:79-219): allocate E*C cars of device state. */
int nascar_create(const NascarConfig* cfg, NascarHandle** out);
void nascar_destroy(NascarHandle* h);
const char* nascar_last_error(void);

/* TrackLoader.load_track + CarPhysics._create_track_walls (src/track_generator.py:305-405,
 * src/car_physics.py:118-339).  Host arrays:
 *   segments: nseg x 13 float64 [type, length, sx, sy, ex, ey, width, curve_angle, curve_radius,
 *             left, start_heading, end_heading, banking]   (type: 0 GRID 1 STARTLINE 2 STRAIGHT 3 FINISHLINE 4 CURVE)
 *   walls:    nwall x 4 float64 [center_x, center_y, angle, half_length] as passed to Box2D
 * The float32 Box2D body transforms (glibc sinf/cosf), fat AABBs and listener keys
 * are derived on the host here.  Returns the track id (>= 0). */
int nascar_add_track(NascarHandle* h, const double* segments, int32_t nseg, double total_length,
                     const double* walls, int32_t nwall);
/* Track build cache (no reference counterpart: the reference rebuilds its walls per CarPhysics, src/car_physics.py:118,
 * and each SubprocVecEnv worker does so on its own, learn/ppo.py:77).  A track's tables (walls, grids and ~0.8 GB of
 * beam lists at 1 m cells, ~2 s of 16 host threads) are shared by every handle of the process; `retain` (default 8)
 * builds stay alive after their last handle closes, most recently used first (0: freed with the last handle).  `dir`
 * (NULL or "" = none, the default) holds on-disk copies of the host tables keyed by the track's arrays and cell size:
 * a process finding one loads it instead of building, one that builds writes it (temporary file + rename), and the
 * processes building one key serialise on a lock file, so the ranks of a node build each track once. */
int nascar_set_track_cache(int32_t retain, const char* dir);
/* Host only (no device): the host tables of one track (arguments as nascar_add_track, plus the beam-list cell size)
 * into the disk cache -- returns 1 if they were already there, 0 if built and written now, < 0 on error (no cache
 * directory set included).  A launcher prebuilds a job's tracks once before its ranks start. */
int nascar_prebuild_track(const double* segments, int32_t nseg, double total_length, const double* walls, int32_t nwall,
                          float beam_cell);

/* per-env track ids (host array of E ints); envs are grouped per track into workgroups (each track's workgroups spread
 * evenly over the workgroup order, so every shard of the sharded rollout holds a share of every track).  A changed id takes
 * effect at that env's next nascar_reset (fresh physics worlds on the new track, as CarEnv.reset recreates
 * CarPhysics, src/car_env.py:375-394); until then the env keeps stepping on its old track.  On a handle that has
 * not been reset, stepped or restored yet the ids apply at once. */
int nascar_set_env_tracks(NascarHandle* h, const int32_t* env_track);

/* Random-track mode, CarEnv(track_file=None) (src/car_env.py:243-303 _select_random_track / _load_random_track,
 * :331-333 and :375-394 in reset; learn/ppo.py:65-78 builds every training env this way).  With ntracks > 0, every
 * reset of an env -- nascar_reset of its mask bit, or the auto-reset inside nascar_step / nascar_step_driven /
 * nascar_rollout -- first draws its next track from the `ntracks` distinct track ids in `tracks` (nascar_add_track ids),
 * uniformly among those that are not its current track (all of them when it is not in the set), and an env whose
 * track changes gets fresh physics worlds there.  Draw k of env e (k counts its draws since seeding, starting at
 * draws[e], NULL = 0) is nascar_track_draw(seeds[e], k, current): a counter hash, reproducible on the host (the
 * reference re-seeds Python's `random` from pid + clock per draw).  The env -> track map, the counters and the
 * workgroup layout live on the device and are updated there (no host synchronisation per step).  ntracks = 0 ends
 * the mode (envs keep their current tracks).  While it is on, nascar_set_env_tracks fails, nascar_rollout runs one
 * shard, and the state snapshot (nascar_get_state) does not carry the env -> track map.  Host arrays; synchronises
 * `stream` once. */
int nascar_set_random_tracks(NascarHandle* h, const int32_t* tracks, int32_t ntracks, const uint64_t* seeds,
                             const int32_t* draws, void* stream);
/* The env -> track ids and the draws taken per env (device int32 [E] each, either may be NULL), on `stream`: the
 * device's in random-track mode, otherwise the host's assignment and zeros. */
int nascar_get_env_tracks(NascarHandle* h, int32_t* env_track, int32_t* draws, void* stream);
/* Host function (no device): the random-track draw for n envs -- out[i] = draw k[i] of seed seeds[i] from an env on
 * track current[i] (-1: none) over tracks[0 .. ntracks). */
int nascar_track_draw(int32_t n, const uint64_t* seeds, const int32_t* k, const int32_t* current, const int32_t* tracks,
                      int32_t ntracks, int32_t* out);

/* SB3 VecEnv glue of the drop-in VecCarEnv (stable_baselines3 Monitor + VecEnv around CarEnv.step, learn/ppo.py:65-78),
 * one launch per step on device buffers:
 * nascar_vec_post: done[e] = terminated | truncated (from env_flags); ep_ret [E*C] float64 += reward, ep_len [E] int64
 *   += 1, their new values copied to snap_ret / snap_len (Monitor's info["episode"] r / l for an env that just ended),
 *   then zeroed for the done envs.
 * nascar_check_actions: *bad (device int32) = 1 if any action is outside the action space (continuous: not in
 *   [-1, 1] or NaN; discrete int32: not in {0..4}) -- CarEnv.step's assert self.action_space.contains(action)
 *   (src/car_env.py:694), read by the caller when it next synchronises. */
int nascar_vec_post(NascarHandle* h, const float* reward, const uint8_t* env_flags, double* ep_ret, int64_t* ep_len,
                    uint8_t* done, double* snap_ret, int64_t* snap_len, void* stream);
int nascar_check_actions(NascarHandle* h, const void* actions, int32_t discrete, int32_t* bad, void* stream);

/* CarEnv.reset (src/car_env.py:316-535) for the envs whose env_mask[e] != 0 (device uint8[E];
 * NULL = all envs).  Writes obs [E*C*38] float32 of the reset envs. */
int nascar_reset(NascarHandle* h, const uint8_t* env_mask, float* obs, void* stream);

/* CarEnv.step (src/car_env.py:678-803) for all E envs.
 *   actions:   continuous: [E*C*2] float32 [throttle_brake, steering] (BaseEnv action space);
 *              discrete:   [E*C] int32 in {0..4} (BaseEnv._discrete_to_continuous, src/base_env.py:227-252)
 *   obs:       [E*C*38] float32 (src/car_env.py:935-946 layout)
 *   reward:    [E*C] float32
 *   car_flags: [E*C] uint8 (bit0 disabled, bit1 just disabled, bit2 collision impulse > 0, bit3 lap completed,
 *              bit7 engine overflow/error)
 *   env_flags: [E] uint8 (bit0 terminated, bit1 truncated, bit3 auto-reset done, bits4-6 termination reason)
 *   auto_reset != 0: envs that terminate/truncate are reset in the same launch; obs then holds the reset
 *              observation and terminal_obs (if non-NULL, [E*C*38]) the final one (SB3 VecEnv convention). */
int nascar_step(NascarHandle* h, const void* actions, int32_t discrete, float* obs, float* reward,
                uint8_t* car_flags, uint8_t* env_flags, int32_t auto_reset, float* terminal_obs, void* stream);

/* nascar_step with the actions of device action source `policy` (0, 1, 3: see nascar_policy_actions) computed on
 * the current obs inside the step launch -- one closed-loop driver step (game/control drivers' loop) without a
 * separate action launch; identical results to nascar_policy_actions(policy, seed, step) + nascar_step. */
int nascar_step_driven(NascarHandle* h, int32_t policy, uint64_t seed, int64_t step, float* obs, float* reward,
                       uint8_t* car_flags, uint8_t* env_flags, int32_t auto_reset, float* terminal_obs, void* stream);

/* Multi-step rollout: `steps` x (device action source on the current obs + CarEnv.step), i.e. the loop
 * of game/control drivers / learn/genetic_trainer.py:225-283 evaluation rollouts (actions from a policy on the
 * previous observation, src/car_env.py:678-803 per step), enqueued in one call with no host synchronisation.
 * Identical results to `steps` calls of nascar_policy_actions(policy, seed, step0 + k) + nascar_step(auto_reset).
 * Default implementation: the envs split into shards stepped on internal streams, forked from `stream` at the
 * start and joined into it at the end (nascar_set_rollout_streams); streams = 0 selects one fused launch.
 *   policy:  0 uniform, 1 BaseController._fallback_control, 3 noisy rule driver (policy 1 with 15 % of the
 *            car-steps uniform) -- see nascar_policy_actions; 2 the SAC actor (nascar_set_actor; sharded
 *            rollout only: each shard runs the actor on its own cars, one shard unless the envs sit in one
 *            track's workgroups in order)
 *   obs:     [E*C*38] float32, in: the current observation, out: the last step's
 *   traj & NASCAR_TRAJ_RECORDS: reward [steps][E*C], car_flags [steps][E*C], env_flags [steps][E] (per-step records);
 *   traj == 0: reward [E*C], car_flags [E*C], env_flags [E] hold the last step's values.
 *   traj & NASCAR_TRAJ_OBS (with NASCAR_TRAJ_RECORDS; sharded rollout only): obs is [steps + 1][E*C*38]; record 0
 *            holds the current observation on entry (read by the action source of step 0) and step k writes
 *            record k + 1 (read by step k + 1) -- a learner's per-step observation buffer, no copies in between.
 * car_flags / env_flags may be NULL.  No terminal observations (auto-reset obs overwrite the final ones). */
#define NASCAR_TRAJ_RECORDS 1
#define NASCAR_TRAJ_OBS 2
int nascar_rollout(NascarHandle* h, int32_t policy, uint64_t seed, int64_t step0, int32_t steps, float* obs,
                   float* reward, uint8_t* car_flags, uint8_t* env_flags, int32_t auto_reset, int32_t traj, void* stream);

/* Rollout implementation (no reference counterpart: a scheduling choice with identical results).
 * streams >= 1: the envs split into `streams` shards of contiguous workgroups, each stepped by per-step launches
 * on its own stream (shard 0 on the caller's), so one shard's slow cars overlap the other shards' work; default:
 * 4, or the process's hardware queues if fewer (GPU_MAX_HW_QUEUES; two shards on one queue run back to back);
 * streams = 0: the fused rollout kernel (all steps in one launch, block barriers between the phases).
 * nascar_get_rollout_streams returns the current setting (-1 for a NULL handle). */
int nascar_set_rollout_streams(NascarHandle* h, int32_t streams);
int nascar_get_rollout_streams(NascarHandle* h);

/* Pipelined rollout (no reference counterpart: a scheduling choice with identical results).  sensor_workgroups > 0:
 * nascar_rollout runs its steps as two persistent kernels -- one workgroup per env group doing the vehicle model, the
 * Box2D step and the env logic K times, and `sensor_workgroups` sensor workgroups taking each group's sensor work from
 * a device queue as the group publishes it -- so every group goes on to its next step as soon as its own sensors are
 * done instead of waiting for the batch's slowest car.  Applies to policies 0, 1, 3 without random tracks, car
 * contact or obs trajectories (the streams setting applies otherwise); 0 turns it off (default).  Every device wait
 * is clock-bounded: nascar_rollout_pipe_status waits for `stream` and returns 1 if a pipelined rollout since the
 * last status call gave up (its results are not valid), 0 if not, -1 on error. */
int nascar_set_rollout_pipe(NascarHandle* h, int32_t sensor_workgroups);
int nascar_rollout_pipe_status(NascarHandle* h, void* stream);

/* Workgroup layout (no reference counterpart: the reference loops over envs and cars one at a time,
 * learn/ppo.py:77 SubprocVecEnv and src/car_env.py:567-570; a scheduling choice with identical results).
 * The one-lane-per-car step kernels run 128-lane workgroups of `epb` whole envs each, epb in [1, 128 / C];
 * epb = 0 restores the automatic choice (128 / C, or fewer envs per workgroup when that leaves fewer than 2
 * workgroups per CU).  May be called at any time; the next launch uses the new layout.
 * nascar_get_envs_per_block returns the current value (-1 for a NULL handle). */
int nascar_set_envs_per_block(NascarHandle* h, int32_t epb);
int nascar_get_envs_per_block(NascarHandle* h);

/* Lanes per car of the distance-sensor kernel (no reference counterpart: DistanceSensor casts its 16 rays one after
 * another, src/distance_sensor.py:93-115): 4 (each lane walks rays r, r + 4, r + 8, r + 12) or 16 (one ray per
 * lane); 0 = automatic (16).  Identical results either way. */
int nascar_set_sensor_lanes(NascarHandle* h, int32_t lanes);

/* Threads per workgroup of the 16-lane distance-sensor kernel (no reference counterpart; src/distance_sensor.py:93-115
 * casts one ray at a time): 64 or 128 (the walks read the track's wall image from global memory; no LDS), 256, 512
 * or 1024 (each workgroup stages the wall image in LDS once for threads / 16 cars); 0 = automatic (128).  Identical
 * results at any size. */
int nascar_set_sensor_block(NascarHandle* h, int32_t threads);

/* Cell size (m) of the distance sensors' beam lists for the tracks added to this handle AFTER the call (host-built
 * per track in nascar_add_track; no reference counterpart -- DistanceSensor ray-casts against every wall,
 * src/distance_sensor.py:93-115).  Default 1 m: ~0.8 GB of device lists and ~2 s of host build
 * per track; 2 m quarters both for slightly longer list walks.  Range [0.5, 8].  Identical results at any size. */
int nascar_set_beam_cell(NascarHandle* h, float meters);

/* Step kernels (no reference counterpart; identical results): enable != 0 (default) runs the vehicle model + Box2D
 * step and the env logic (disable rules, lap timer, obs[0:22], rewards, termination, auto-reset;
 * src/car_env.py:537-803, 805-1158) as one launch per step, each workgroup starting its envs' logic when its own cars'
 * Box2D steps are done; 0 runs them as two launches (model_kernel, logic_kernel).  nascar_get_fused_logic returns the
 * current setting (-1 for a NULL handle). */
int nascar_set_fused_logic(NascarHandle* h, int32_t enable);
int nascar_get_fused_logic(NascarHandle* h);

/* Profiling hook (no reference counterpart; bench.py's per-kernel roofline): events = 4 caller-created timing
 * events (hipEvent_t), recorded by every following whole-grid step (nascar_step / nascar_step_driven) on its
 * stream before model_kernel, after model_kernel, after logic_kernel and after the sensor launch; n = 0 stops.
 * The events stay owned by the caller and must outlive their use. */
int nascar_set_step_events(NascarHandle* h, void* const* events, int32_t n);

/* Info builder (src/car_env.py:1160-1227, src/lap_timer.py:354-372): per-car float64 [E*C*N_INFO]
 * (field order: nascargymnasium_amd/_lib.py INFO_FIELDS) written to a device buffer. */
int nascar_get_info(NascarHandle* h, double* info, void* stream);

/* BUILD-ONLY EXTENSION, no reference counterpart (each reference car has its own b2World, so cars never touch):
 * enable != 0 makes the cars of an env collide -- staggered start grid (rows of 2, 8 m apart), and after each
 * Box2D step a frictionless central impulse (restitution 0.25) between overlapping, closing car boxes, counted in
 * the cars' collision impulse (damage / impact disables).  Default 0 (reference behaviour); parity runs with 0.
 * Takes effect from the next reset (start grid) and step. */
int nascar_set_car_contact(NascarHandle* h, int32_t enable);

/* Car.velocity_history for Car.validate_performance (src/car.py:173, 384-386, 1060-1098): enable != 0 keeps
 * every car's speed after each step in a 600-sample window on the device (VH_RING x N float32, outside the
 * state arena, so snapshots do not carry it) and nascar_get_info reports perf_count / perf_max_speed /
 * perf_first_fast; 0 frees it (the info fields then read -1 / 0 / -1).  Off by default. */
int nascar_set_perf_history(NascarHandle* h, int32_t enable, void* stream);

/* Raw state snapshot / restore (checkpointing and state-injection parity tests). */
int64_t nascar_state_bytes(NascarHandle* h);
int nascar_get_state(NascarHandle* h, void* dst_device, void* stream);
int nascar_set_state(NascarHandle* h, const void* src_device, void* stream);

/* Device action sources:
 *   policy 0: counter-based uniform U[-1,1]^2 (key = seed, car, step)
 *   policy 1: BaseController._fallback_control (game/control/base_controller.py:39-103) from obs
 *   policy 2: the SAC actor loaded with nascar_set_actor, deterministic (SACController.control,
 *             game/control/sac_control_class.py:80-115) from obs
 *   policy 3: policy 1 with its action replaced by policy 0's draw on 15 % of the car-steps (counter hash) */
int nascar_policy_actions(NascarHandle* h, int32_t policy, uint64_t seed, int64_t step, const float* obs,
                          float* actions, void* stream);

/* SB3 SAC MlpPolicy actor weights (PyTorch layouts, host float32): w1 [256][38], b1 [256],
 * w2 [256][256], b2 [256], w3 = mu.weight [2][256], b3 = mu.bias [2]  (obs_dim 38, hidden 256,
 * act_dim 2; other shapes are rejected).  Replaces SAC.load + policy.predict
 * (game/control/sac_control_class.py:48-115) with one fused actor kernel: float32 by default, the bf16-operand
 * MFMA kernel on request (nascar_set_actor_precision). */
int nascar_set_actor(NascarHandle* h, const float* w1, const float* b1, const float* w2, const float* b2,
                     const float* w3, const float* b3, int32_t obs_dim, int32_t hidden, int32_t act_dim);
/* Actor arithmetic for policy 2 and nascar_actor_forward: 1 (default) = float32 throughout (the reference's
 * model.predict precision; <= 1e-5 on the reference's sac_1235 checkpoint, tests/test_gpu_actor.py), 0 = the
 * bf16-operand MFMA kernel (fp32 accumulation; ~8x faster: 16.2 vs 135 us at 81 920 observations, max |delta action|
 * 0.40 on sac_1235). */
int nascar_set_actor_precision(NascarHandle* h, int32_t fp32);
/* The loaded actor on any device batch: obs [n][38] float32 -> actions [n][2] float32 (both 8-byte aligned). */
int nascar_actor_forward(NascarHandle* h, const float* obs, int32_t n, float* actions, void* stream);

/* Test hook: the device re-implementation of glibc sinf/cosf used for b2Rot::Set
 * (device pointers, n floats).  Parity tests compare it with the host libm. */
int nascar_debug_sincosf(const float* x, float* s, float* c, int32_t n, void* stream);

/* Test hook: sensors only.  poses: device float32 [E*C*3] (x, y, angle) per car, written into the sensor
 * hand-off; impl 1 = beam-list ray kernel (the step's default), 0 = wall-group kernel; writes the 16
 * DistanceSensor values obs[n*38 + 22 .. 37] (src/distance_sensor.py:71-117, src/car_env.py:946). */
int nascar_debug_sensors(NascarHandle* h, const float* poses, float* obs, int32_t impl, void* stream);

/* Test hook: the workgroup layout the next launch uses (block map; prepare()d first) copied into caller device buffers,
 * blk_track [cap_blocks] and blk_env [cap_blocks * envs per workgroup] int32; returns the number of workgroups launched
 * (random-track mode: those past the last track's are empty, track -1), or < 0 on error. */
int nascar_debug_block_map(NascarHandle* h, int32_t* blk_track, int32_t* blk_env, int32_t cap_blocks, void* stream);

#ifdef __cplusplus
}
#endif
#endif
