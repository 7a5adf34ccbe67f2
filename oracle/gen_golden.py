"""Generate the committed golden fixtures under tests/golden/ (run in the build
container only; needs /root/reference, never runs on the GPU box).

TEST INFRASTRUCTURE ONLY.  The reference's third-party deps (Box2D, gymnasium,
pygame) are absent here, so they are replaced by stub modules:

* ``pygame``  -- permissive no-op module (only constants/fonts are touched on the
  headless path: src/constants/ui.py:3,116-117, src/observation_visualizer_optimized.py:93).
* ``gymnasium`` -- Env base + spaces restated from gymnasium==0.29.1.
* ``Box2D``  -- a recording stub whose dynamic-body worlds delegate to the
  oracle's Box2D restatement (oracle/b2_oracle.c via liboracle.so ``hb_*``).

With that, the reference's OWN ``CarEnv``/``Car``/``TyreManager``/``LapTimer``/
``CarPhysics`` Python runs unchanged ("hybrid oracle") and
its outputs become the golden vectors that pin the C oracle's restatement of
everything except the Box2D internals.

Usage:  python oracle/gen_golden.py [--ref /root/reference] [--out tests/golden]
"""
import argparse
import ctypes
import os
import sys
import types

import numpy as np

# the reference's modules are imported from /root/reference (read-only): never leave bytecode there
sys.dont_write_bytecode = True

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_lib  # noqa: E402

f32 = np.float32


# ----------------------------------------------------------------- pygame stub
class _Any:
    def __init__(self, *a, **k):
        pass

    def __call__(self, *a, **k):
        return _Any()

    def __getattr__(self, name):
        return _Any()

    def __iter__(self):
        return iter(())

    def __bool__(self):
        return False


class _PygameModule(types.ModuleType):
    def __getattr__(self, name):
        if name.startswith("K_"):
            return 1000 + sum(ord(ch) for ch in name)
        return _Any()


def make_pygame():
    pg = _PygameModule("pygame")
    for i in range(10):
        setattr(pg, f"K_{i}", 48 + i)
    pg.font = _Any()
    pg.get_init = lambda: False
    return pg


# -------------------------------------------------------------- gymnasium stub
def make_gymnasium():
    gym = types.ModuleType("gymnasium")
    spaces = types.ModuleType("gymnasium.spaces")

    class Env:
        metadata = {}

        def reset(self, seed=None, options=None):
            return None

    class Box:
        def __init__(self, low, high, shape=None, dtype=np.float32):
            self.dtype = np.dtype(dtype)
            self.shape = tuple(shape) if shape is not None else np.shape(low)
            self.low = np.broadcast_to(np.asarray(low, self.dtype), self.shape)
            self.high = np.broadcast_to(np.asarray(high, self.dtype), self.shape)

        def contains(self, x):
            if not isinstance(x, np.ndarray):
                try:
                    x = np.asarray(x, dtype=self.dtype)
                except (ValueError, TypeError):
                    return False
            return bool(np.can_cast(x.dtype, self.dtype) and x.shape == self.shape
                        and np.all(x >= self.low) and np.all(x <= self.high))

    class Discrete:
        def __init__(self, n, start=0):
            self.n, self.start = n, start

        def contains(self, x):
            if isinstance(x, int):
                v = np.int64(x)
            elif isinstance(x, (np.generic, np.ndarray)) and np.issubdtype(x.dtype, np.integer) and x.shape == ():
                v = np.int64(x)
            else:
                return False
            return bool(self.start <= v < self.start + self.n)

    class MultiDiscrete:
        def __init__(self, nvec):
            self.nvec = np.asarray(nvec, np.int64)
            self.shape = self.nvec.shape

        def contains(self, x):
            if isinstance(x, (list, tuple)):
                x = np.array(x)
            return bool(isinstance(x, np.ndarray) and x.shape == self.shape and x.dtype != object
                        and np.all(0 <= x) and np.all(x < self.nvec))

    spaces.Box, spaces.Discrete, spaces.MultiDiscrete = Box, Discrete, MultiDiscrete
    gym.Env, gym.spaces = Env, spaces
    return gym, spaces


# -------------------------------------------------------------------- Box2D stub
class Vec(tuple):
    """b2Vec2 as pybox2d hands it to Python: float32 components."""

    def __new__(cls, x, y):
        return tuple.__new__(cls, (float(f32(x)), float(f32(y))))

    @property
    def x(self):
        return self[0]

    @property
    def y(self):
        return self[1]

    @property
    def length(self):  # b2Vec2::Length in float32
        x, y = f32(self[0]), f32(self[1])
        return float(np.sqrt(f32(x * x + y * y)))


def make_box2d(hb_env):
    L = oracle_lib.lib()
    vp = ctypes.c_void_p
    L.hb_world_create.restype = vp
    L.hb_world_create.argtypes = [vp, ctypes.c_float, ctypes.c_float, ctypes.c_float]
    L.hb_apply_force.argtypes = [vp] + [ctypes.c_float] * 4
    L.hb_apply_force_center.argtypes = [vp] + [ctypes.c_float] * 2
    L.hb_apply_torque.argtypes = [vp, ctypes.c_float]
    BEGIN = ctypes.CFUNCTYPE(None, ctypes.c_int, ctypes.c_float, ctypes.c_float)
    END = ctypes.CFUNCTYPE(None, ctypes.c_int)
    POST = ctypes.CFUNCTYPE(None, ctypes.c_int, ctypes.c_float, ctypes.c_float)
    L.hb_step.argtypes = [vp, vp, ctypes.c_float, ctypes.c_int, ctypes.c_int, BEGIN, END, POST]
    L.hb_get.argtypes = [vp, ctypes.POINTER(ctypes.c_float)]
    L.hb_set_transform.argtypes = [vp, vp] + [ctypes.c_float] * 3
    L.hb_set_velocity.argtypes = [vp] + [ctypes.c_float] * 2
    L.hb_set_angular_velocity.argtypes = [vp, ctypes.c_float]

    wd, wf = hb_env.walls()        # oracle wall table (float part used for the query/raycast stubs)

    B = types.ModuleType("Box2D")
    B.b2_dynamicBody, B.b2_staticBody, B.b2_kinematicBody = 2, 0, 1

    class _Base:
        def __init__(self, *a, **k):
            pass

    B.b2RayCastCallback = B.b2ContactListener = B.b2QueryCallback = _Base
    B.b2Body = type("b2Body", (), {})

    class b2BodyDef:
        def __init__(self):
            self.type, self.position, self.angle = 0, (0.0, 0.0), 0.0

    class b2PolygonShape:
        def __init__(self):
            self.hx = self.hy = 0.0

        def SetAsBox(self, hx, hy):
            self.hx, self.hy = float(f32(hx)), float(f32(hy))
            self.dhx, self.dhy = hx, hy

        @property
        def vertexCount(self):
            return 4

        @property
        def vertices(self):
            hx, hy = self.hx, self.hy
            return [Vec(-hx, -hy), Vec(hx, -hy), Vec(hx, hy), Vec(-hx, hy)]

        def TestPoint(self, xf, p):  # b2PolygonShape::TestPoint in float32
            (px, py), (s, c) = xf
            dx, dy = f32(f32(p[0]) - f32(px)), f32(f32(p[1]) - f32(py))
            lx = f32(f32(c * dx) + f32(s * dy))
            ly = f32(f32(-s * dx) + f32(c * dy))
            hx, hy = f32(self.hx), f32(self.hy)
            verts = [(-hx, -hy), (hx, -hy), (hx, hy), (-hx, hy)]
            norms = [(f32(0), f32(-1)), (f32(1), f32(0)), (f32(0), f32(1)), (f32(-1), f32(0))]
            for (vx, vy), (nx, ny) in zip(verts, norms):
                d = f32(f32(nx * f32(lx - vx)) + f32(ny * f32(ly - vy)))
                if d > 0:
                    return False
            return True

    B.b2PolygonShape = b2PolygonShape

    def b2Mul(xf, v):
        (px, py), (s, c) = xf
        x, y = f32(v[0]), f32(v[1])
        return Vec(f32(f32(f32(c * x) - f32(s * y)) + f32(px)), f32(f32(f32(s * x) + f32(c * y)) + f32(py)))

    B.b2Mul = b2Mul

    class _Filter:
        categoryBits = maskBits = 0

    class b2FixtureDef:
        def __init__(self):
            self.shape, self.density, self.friction, self.restitution = None, 0, 0, 0
            self.filter = _Filter()

    class b2MassData:
        mass, center, I = 0.0, (0, 0), 0.0

    class b2AABB:
        lowerBound = upperBound = (0, 0)

    B.b2BodyDef, B.b2FixtureDef, B.b2MassData, B.b2AABB = b2BodyDef, b2FixtureDef, b2MassData, b2AABB

    class Fixture:
        def __init__(self, body, fd):
            self.body, self.shape, self.userData = body, fd.shape, None

    class StaticBody:
        def __init__(self, world, bd, index):
            self.world, self.index = world, index
            self.def_position, self.def_angle = tuple(bd.position), bd.angle
            self.position = Vec(*bd.position)
            self.angle = float(f32(bd.angle))
            self.userData = None
            self.fixture = None
            row = wf[index]
            self.transform = ((float(row[0]), float(row[1])), (float(row[5]), float(row[6])))

        def CreateFixture(self, fd):
            self.fixture = Fixture(self, fd)
            return self.fixture

    class CarBody:
        def __init__(self, world, bd):
            self.world = world
            self.w = L.hb_world_create(hb_env.h, f32(bd.position[0]), f32(bd.position[1]), f32(bd.angle))
            self.userData = None
            self.contacts = []

        def _st(self):
            o = (ctypes.c_float * 8)()
            L.hb_get(self.w, o)
            return list(o)

        def CreateFixture(self, fd):
            return Fixture(self, fd)

        massData = property(lambda self: None, lambda self, v: None)

        @property
        def position(self):
            s = self._st()
            return Vec(s[0], s[1])

        @position.setter
        def position(self, v):
            L.hb_set_transform(hb_env.h, self.w, f32(v[0]), f32(v[1]), f32(self._st()[2]))

        @property
        def angle(self):
            return float(f32(self._st()[2]))

        @angle.setter
        def angle(self, a):
            s = self._st()
            L.hb_set_transform(hb_env.h, self.w, f32(s[0]), f32(s[1]), f32(a))

        @property
        def linearVelocity(self):
            s = self._st()
            return Vec(s[3], s[4])

        @linearVelocity.setter
        def linearVelocity(self, v):
            L.hb_set_velocity(self.w, f32(v[0]), f32(v[1]))

        @property
        def angularVelocity(self):
            return float(f32(self._st()[5]))

        @angularVelocity.setter
        def angularVelocity(self, a):
            L.hb_set_angular_velocity(self.w, f32(a))

        def GetWorldVector(self, v):
            s = self._st()
            qs, qc = f32(s[6]), f32(s[7])
            x, y = f32(v[0]), f32(v[1])
            return Vec(f32(f32(qc * x) - f32(qs * y)), f32(f32(qs * x) + f32(qc * y)))

        def GetWorldPoint(self, v):
            s = self._st()
            return b2Mul(((s[0], s[1]), (s[6], s[7])), v)

        def ApplyForce(self, f, p, wake):
            L.hb_apply_force(self.w, f32(f[0]), f32(f[1]), f32(p[0]), f32(p[1]))

        def ApplyForceToCenter(self, f, wake):
            L.hb_apply_force_center(self.w, f32(f[0]), f32(f[1]))

        def ApplyTorque(self, t, wake):
            L.hb_apply_torque(self.w, f32(t))

    class _WM:
        def __init__(self, n):
            self.normal = Vec(*n)
            self.points = [Vec(0, 0)]

    class _Contact:
        def __init__(self, car, wall, normal=None):
            self.fixtureA = types.SimpleNamespace(body=car)
            self.fixtureB = types.SimpleNamespace(body=wall)
            if normal is not None:
                self.worldManifold = _WM(normal)

    class b2World:
        def __init__(self, gravity=(0, 0), **kw):
            self.car, self.walls, self.contactListener = None, [], None

        def CreateBody(self, bd):
            if bd.type == B.b2_dynamicBody:
                self.car = CarBody(self, bd)
                return self.car
            b = StaticBody(self, bd, len(self.walls))
            self.walls.append(b)
            return b

        @property
        def bodies(self):
            return [self.car] + self.walls

        def Step(self, dt, vi, pi):
            lis = self.contactListener

            def begin(j, nx, ny):
                lis.BeginContact(_Contact(self.car, self.walls[j], (nx, ny)))

            def end(j):
                lis.EndContact(_Contact(self.car, self.walls[j]))

            def post(count, n0, n1):
                imp = types.SimpleNamespace(normalImpulses=tuple([float(n0), float(n1)][:count]))
                lis.PostSolve(_Contact(self.car, None), imp)

            cb = (BEGIN(begin), END(end), POST(post))
            L.hb_step(hb_env.h, self.car.w, f32(dt), vi, pi, *cb)

        def RayCast(self, callback, p1, p2):
            fr = L.or_raycast(hb_env.h, f32(p1[0]), f32(p1[1]), f32(p2[0]), f32(p2[1]))
            if fr >= 0:
                callback.ReportFixture(self.walls[0].fixture, Vec(0, 0), Vec(0, 0), float(fr))

        def QueryAABB(self, callback, aabb):
            lo, hi = (f32(aabb.lowerBound[0]), f32(aabb.lowerBound[1])), (f32(aabb.upperBound[0]), f32(aabb.upperBound[1]))
            for j, b in enumerate(self.walls):
                r = wf[j]
                if (lo[0] - r[9] > 0 or lo[1] - r[10] > 0 or r[7] - hi[0] > 0 or r[8] - hi[1] > 0):
                    continue
                if callback.ReportFixture(b.fixture) is False:
                    return

    B.b2World = b2World
    return B


def install_stubs(hb_env):
    sys.modules["pygame"] = make_pygame()
    gym, spaces = make_gymnasium()
    sys.modules["gymnasium"] = gym
    sys.modules["gymnasium.spaces"] = spaces
    sys.modules["Box2D"] = make_box2d(hb_env)


def purge_reference_modules():
    for k in list(sys.modules):
        if k == "src" or k.startswith("src."):
            del sys.modules[k]


# ------------------------------------------------------------- driver policies
class RuleDriver:
    """BaseController._fallback_control (game/control/base_controller.py:39-103),
    imported from the reference itself."""

    def __init__(self, ref):
        sys.path.insert(0, os.path.join(ref, "game", "control"))
        from base_controller import BaseController  # noqa: E402
        self.c = BaseController()

    def __call__(self, obs):
        return self.c._fallback_control(obs)


INFO_KEYS = ["lap_count", "last_lap_time", "best_lap_time", "is_timing", "current_lap_time",
             "total_distance_traveled", "car_speed_ms", "on_track", "disabled", "cumulative_reward",
             "cumulative_impact_force"]


def car_info_row(ci):
    lt = ci.get("lap_timing", {})
    g = lambda v: np.nan if v is None else float(v)  # noqa: E731
    return [g(lt.get("lap_count")), g(lt.get("last_lap_time")), g(lt.get("best_lap_time")), g(lt.get("is_timing")),
            g(lt.get("current_lap_time")), g(lt.get("total_distance_traveled")), g(ci.get("car_speed_ms")),
            g(ci.get("on_track")), g(ci.get("disabled")), g(ci.get("cumulative_reward")), g(ci.get("cumulative_impact_force"))]


PERF_KEYS = ["current_max_speed", "estimated_0_100_time", "performance_valid"]   # Car.validate_performance


def perf_row(p):
    return [float(p.get(k, np.nan)) for k in PERF_KEYS]


REASONS = {None: 0, "all_cars_disabled": 1, "time_limit": 3, "truncated": 4}


def reason_code(r):
    if r is None:
        return 0
    if r.startswith("all_active_cars_low_reward"):
        return 2
    return REASONS[r]


DISCRETE_P = [0.1, 0.5, 0.1, 0.15, 0.15]   # Discrete(5) draws: mostly throttle, some braking / steering


def policy_action(mode, k, driver, obs, rng):
    """one car's action for policy `mode` (a name, or a tuple (name, *params)) at step k"""
    name, par = (mode[0], mode[1:]) if isinstance(mode, tuple) else (mode, ())
    if name == "rule":
        return driver(obs)
    if name == "rule_noisy":
        a = driver(obs)
        return rng.uniform(-1, 1, 2).astype(np.float32) if rng.random() < 0.15 else a
    if name == "rule_bias":      # full throttle, steering biased toward the outer wall (grinds it: damage)
        a = driver(obs)
        return np.array([1.0, min(1.0, float(a[1]) + par[0])], np.float32)
    if name == "uturn":          # (t0, t1, throttle, steer): turn round inside (t0, t1), then the rule driver
        a = driver(obs)
        return np.array([par[2], par[3]], np.float32) if par[0] < k < par[1] else a
    if name == "spin":           # (steer, period): throttle + steer, then full brake, periodically
        on = k % par[1] < 0.6 * par[1]
        return np.array([1.0 if on else -1.0, par[0] if on else 0.0], np.float32)
    if name == "random":
        return rng.uniform(-1, 1, 2).astype(np.float32)
    if name == "throttle":
        return np.array([1.0, 0.0], np.float32)
    if name == "throttle_left":
        return np.array([1.0, -0.3 if k > 100 else 0.0], np.float32)
    if name == "idle":
        return np.array([0.0, 0.0], np.float32)
    if name == "brake_back":
        return np.array([-1.0 if k % 200 < 120 else 0.6, 0.8 if k % 300 < 100 else -0.2], np.float32)
    if name == "discrete":
        return int(rng.choice(5, p=DISCRETE_P))
    raise ValueError(mode)


def run_scenario(ref, name, track, C, steps, policy, reset_on_lap=False, reset_at=(), seed=0, discrete=False,
                 start_position=None, start_angle=0.0):
    """Run the REFERENCE CarEnv (stub Box2D -> oracle Box2D) and record everything."""
    track_path = os.path.join(ref, "tracks", track)
    hb = oracle_lib.OracleEnv(track_path, 1, 1)
    install_stubs(hb)
    purge_reference_modules()
    sys.path.insert(0, ref)
    import contextlib
    import io
    with contextlib.redirect_stdout(io.StringIO()):
        from src.car_env import CarEnv
        env = CarEnv(render_mode=None, track_file=track_path, num_cars=C, reset_on_lap=reset_on_lap,
                     discrete_action_space=discrete, start_position=start_position, start_angle=start_angle)
        obs, info = env.reset()
    rng = np.random.default_rng(seed)
    drivers = [RuleDriver(ref) for _ in range(C)]
    rec = {k: [] for k in ["actions", "obs", "rewards", "terminated", "truncated", "reason", "sim_time", "info", "reset",
                           "perf", "physics"]}
    obs = obs.reshape(C, 38)
    rec["obs0"] = obs.copy()
    for k in range(steps):
        acts = []
        for i in range(C):
            a = policy_action(policy[i % len(policy)], k, drivers[i], obs[i], rng)
            acts.append(a if discrete else np.clip(np.asarray(a, np.float32), -1, 1))
        acts = np.array(acts, np.int32) if discrete else np.stack(acts).astype(np.float32)
        did_reset = k in reset_at
        with contextlib.redirect_stdout(io.StringIO()):
            if did_reset:
                obs, info = env.reset()
                obs = obs.reshape(C, 38)
                rec["actions"].append(np.zeros(C, np.int32) if discrete else np.zeros((C, 2), np.float32))
                rec["obs"].append(obs.copy()); rec["rewards"].append(np.zeros(C, np.float32))
                rec["terminated"].append(False); rec["truncated"].append(False)
            else:
                if discrete:
                    a_in = int(acts[0]) if C == 1 else acts.astype(np.int64)
                else:
                    a_in = acts[0] if C == 1 else acts
                obs, rew, term, trunc, info = env.step(a_in)
                obs = obs.reshape(C, 38)
                rec["actions"].append(acts); rec["obs"].append(obs.copy())
                rec["rewards"].append(np.asarray(rew, np.float32).reshape(C))
                rec["terminated"].append(bool(term)); rec["truncated"].append(bool(trunc))
        rec["reset"].append(did_reset)
        rec["reason"].append(reason_code(env.termination_reason))
        rec["sim_time"].append(info["simulation_time"])
        rec["info"].append([car_info_row(ci) for ci in info["cars"]])
        rec["perf"].append([perf_row(ci.get("performance", {})) for ci in info["cars"]])
        rec["physics"].append([[float(p["physics_steps"]), float(p["simulation_time"]), float(p["average_fps"]),
                                float(p["bodies_in_world"])] for p in info["physics"]])
    sys.path.remove(ref)
    n = len(rec["obs"])
    keep = np.arange(n) if n <= 4000 else np.unique(np.r_[np.arange(0, n, 50), np.arange(n - 20, n)])
    out = dict(track=np.array(track), C=np.array(C), reset_on_lap=np.array(reset_on_lap), discrete=np.array(discrete),
               actions=np.array(rec["actions"], np.int32 if discrete else np.float32),
               obs=np.array(rec["obs"], np.float32)[keep],
               obs_steps=keep,
               rewards=np.array(rec["rewards"], np.float32), terminated=np.array(rec["terminated"]),
               truncated=np.array(rec["truncated"]), reason=np.array(rec["reason"], np.int32),
               sim_time=np.array(rec["sim_time"]), info=np.array(rec["info"], np.float64)[keep],
               reset=np.array(rec["reset"]), obs0=rec["obs0"],
               perf=np.array(rec["perf"], np.float64)[keep], physics=np.array(rec["physics"], np.float64)[keep])
    if start_position is not None or start_angle != 0.0:     # CarEnv(start_position=, start_angle=) (src/car_env.py:82-83)
        out["start_position"] = np.array(start_position if start_position is not None else (np.nan, np.nan), np.float64)
        out["start_angle"] = np.array(start_angle, np.float64)
    return out


def track_tables(ref, track):
    """Reference Track + wall builder tables (TrackLoader + CarPhysics._create_track_walls)."""
    track_path = os.path.join(ref, "tracks", track)
    hb = oracle_lib.OracleEnv(track_path, 1, 1)
    install_stubs(hb)
    purge_reference_modules()
    sys.path.insert(0, ref)
    from src.track_generator import TrackLoader
    from src.car import Car
    from src.car_physics import CarPhysics
    t = TrackLoader().load_track(track_path)
    types_ = {"GRID": 0, "STARTLINE": 1, "STRAIGHT": 2, "FINISHLINE": 3, "CURVE": 4}
    segs = np.array([[types_[s.segment_type], s.length, s.start_position[0], s.start_position[1], s.end_position[0],
                      s.end_position[1], s.width, s.curve_angle, s.curve_radius, 1.0 if s.curve_direction == "LEFT" else 0.0,
                      s.start_heading, s.end_heading, s.banking_angle] for s in t.segments], np.float64)
    cp = CarPhysics(Car(world=None), t)
    walls = np.array([[b.def_position[0], b.def_position[1], b.def_angle, b.fixture.shape.dhx, b.fixture.shape.dhy]
                      for b in cp.world.walls], np.float64)
    keys = np.array([f"wall_{b.position.x:.1f}_{b.position.y:.1f}" for b in cp.world.walls])
    sys.path.remove(ref)
    return dict(segments=segs, total_length=np.array(t.total_length), walls=walls, keys=keys,
                has_banking=np.array(cp._track_has_banking()))


SCENARIOS = [
    # name, track, cars, steps, per-car policy, reset_on_lap, reset_at
    ("daytona_mixed", "daytona.track", 3, 1500, ["rule", "random", "throttle"], False, ()),
    ("daytona_crash", "daytona.track", 2, 1300, ["throttle_left", "brake_back"], False, (700,)),
    ("talladega_noisy", "talladega.track", 2, 700, ["rule_noisy", "throttle_left"], False, ()),
    ("michigan_banked", "michigan.track", 2, 700, ["rule", "brake_back"], False, (350,)),
    ("martinsville_lap", "martinsville.track", 2, 3700, ["rule", "rule_noisy"], True, ()),
    ("daytona_long", "daytona.track", 1, 10810, ["rule"], False, ()),
    ("nascar2_seam", "nascar2.track", 1, 600, ["rule_noisy"], False, ()),
    ("trioval_idle", "trioval.track", 2, 720, ["idle", "random"], False, ()),
    # round 2: every termination reason and disable branch, discrete actions, 10 cars, all 8 tracks
    ("martinsville_all_idle", "martinsville.track", 3, 660, ["idle"], False, ()),                 # reason 1
    ("daytona_low_reward", "daytona.track", 2, 900, [("spin", 0.35, 300), ("spin", 0.5, 180)], False, ()),  # reason 2
    ("daytona_damage", "daytona.track", 2, 3000, [("rule_bias", 0.1), "rule"], False, ()),     # cumulative damage
    ("nascar_backward", "nascar.track", 2, 900, ["rule", ("uturn", 100, 200, 0.3, 1.0)], False, ()),  # backward
    ("nascar_banked_discrete", "nascar_banked.track", 3, 900, ["discrete"], False, (), {"discrete": True}),
    ("michigan_discrete1", "michigan.track", 1, 700, ["discrete"], False, (), {"discrete": True}),
    ("talladega_10car", "talladega.track", 10, 1500, ["rule", "rule_noisy", "random", "throttle", "throttle_left",
                                                      "brake_back", "idle", "rule_noisy", ("rule_bias", 0.2), "rule"],
     False, (900,)),
    # round 3: non-default CarEnv(start_position=, start_angle=) (src/car_env.py:82-83,114-115,391,398)
    ("nascar_start_pose", "nascar.track", 2, 1200, ["rule", "rule_noisy"], False, (600,),
     {"start_position": (150.0, 4.0), "start_angle": 0.15}),
    ("daytona_start_reversed", "daytona.track", 2, 900, ["rule", "rule_noisy"], False, (450,),
     {"start_position": (60.0, -3.0), "start_angle": 3.0}),
]


NEW = {"martinsville_all_idle", "daytona_low_reward", "daytona_damage", "nascar_backward", "nascar_banked_discrete",
       "michigan_discrete1", "talladega_10car", "nascar_start_pose", "daytona_start_reversed"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--out", default=os.path.join(ROOT, "tests", "golden"))
    ap.add_argument("--only", default=None)
    args = ap.parse_args()
    os.makedirs(args.out, exist_ok=True)
    oracle_lib.build()
    tracks = sorted(f for f in os.listdir(os.path.join(args.ref, "tracks")) if f.endswith(".track"))
    if args.only in (None, "tracks"):
        allt = {}
        for tr in tracks:
            d = track_tables(args.ref, tr)
            for k, v in d.items():
                allt[f"{tr[:-6]}__{k}"] = v
        np.savez_compressed(os.path.join(args.out, "tracks.npz"), **allt)
        print("tracks.npz", len(tracks))
    for name, track, C, steps, pol, rol, rat, *extra in SCENARIOS:
        if args.only not in (None, name) and not (args.only == "new" and extra is not None and name in NEW):
            continue
        d = run_scenario(args.ref, name, track, C, steps, pol, rol, rat, **(extra[0] if extra else {}))
        np.savez_compressed(os.path.join(args.out, f"env_{name}.npz"), **d)
        term = d["terminated"].nonzero()[0]
        print(name, "steps", len(d["obs"]), "laps", np.nanmax(d["info"][..., 0]), "disabled", d["info"][-1, :, 8],
              "first-term", term[:1], "reasons", np.unique(d["reason"]))


if __name__ == "__main__":
    main()
