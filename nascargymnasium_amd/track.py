"""Track pipeline: ``.track`` file -> segment table + Box2D wall-box table.

Host-side, float64 Python like the reference (so the tables are bit-identical):

* ``load_track`` restates ``TrackLoader.load_track`` / ``Track.add_segment``
  (reference src/track_generator.py:66-115, 305-405), same errors
  (FileNotFoundError / ValueError with the reference's messages).
* ``build_walls`` restates ``CarPhysics._create_track_walls`` and helpers
  (src/car_physics.py:118-339): 1 m-thick boxes along straights and along the
  1-degree chords of curves -- the geometry the sensors and contacts see
  (src/track_boundary.py is render-only and NOT used).

The float32 Box2D transforms, fat AABBs and listener keys are derived from these
tables inside libnascar.so (nascar_add_track) with the host libm, as Box2D does.
"""
import math
import os
from dataclasses import dataclass, field
from typing import List, Tuple

import numpy as np

DEFAULT_TRACK_WIDTH = 20.0     # src/constants/track.py:4
DEFAULT_GRID_LENGTH = 100.0    # :5
STARTLINE_LENGTH = 5.0         # :6
FINISHLINE_LENGTH = 5.0        # :7
TRACK_WALL_THICKNESS = 1.0     # :16
PHYSICS_CURVE_DEGREES_PER_SEGMENT = 1.0   # src/constants/physics.py:23
PHYSICS_CURVE_MIN_SEGMENTS = 8
PHYSICS_CURVE_MAX_SEGMENTS = 180
SEG_TYPES = {"GRID": 0, "STARTLINE": 1, "STRAIGHT": 2, "FINISHLINE": 3, "CURVE": 4}

TRACKS_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tracks")


def track_path(name: str) -> str:
    """'daytona' / 'daytona.track' / a path -> path of the .track file."""
    if os.path.exists(name):
        return name
    base = name if name.endswith(".track") else name + ".track"
    p = os.path.join(TRACKS_DIR, os.path.basename(base))
    return p


def available_tracks() -> List[str]:
    return sorted(os.path.join(TRACKS_DIR, f) for f in os.listdir(TRACKS_DIR) if f.endswith(".track"))


@dataclass
class TrackSegment:
    """src/track_generator.py:13-40"""
    segment_type: str
    length: float
    start_position: Tuple[float, float]
    end_position: Tuple[float, float]
    width: float
    curve_angle: float = 0.0
    curve_radius: float = 0.0
    curve_direction: str = ""
    start_heading: float = 0.0
    end_heading: float = 0.0
    banking_angle: float = 0.0


@dataclass
class Track:
    """src/track_generator.py:43-115"""
    width: float = DEFAULT_TRACK_WIDTH
    segments: List[TrackSegment] = field(default_factory=list)
    total_length: float = 0.0
    current_position: Tuple[float, float] = (0.0, 0.0)
    current_heading: float = 0.0
    name: str = ""

    def add_segment(self, segment_type, length, curve_angle=0.0, curve_radius=0.0, curve_direction="", banking_angle=0.0):
        start_pos, start_heading = self.current_position, self.current_heading
        if curve_angle == 0.0:
            end_heading = start_heading
            hr = math.radians(start_heading)
            end_pos = (start_pos[0] + length * math.cos(hr), start_pos[1] + length * math.sin(hr))
        else:
            segment_type = "CURVE"
            shr = math.radians(start_heading)
            car = math.radians(curve_angle)
            turn = 1.0 if curve_direction == "LEFT" else -1.0
            perp = shr + turn * math.pi / 2
            cx = start_pos[0] + curve_radius * math.cos(perp)
            cy = start_pos[1] + curve_radius * math.sin(perp)
            end_heading = start_heading + turn * curve_angle
            a0 = shr - turn * math.pi / 2
            a1 = a0 + turn * car
            end_pos = (cx + curve_radius * math.cos(a1), cy + curve_radius * math.sin(a1))
            length = abs(curve_radius * math.radians(curve_angle))
        self.segments.append(TrackSegment(segment_type, length, start_pos, end_pos, self.width, curve_angle,
                                          curve_radius, curve_direction, start_heading, end_heading, banking_angle))
        self.total_length += length
        self.current_position, self.current_heading = end_pos, end_heading

    def get_total_track_length(self) -> float:
        return self.total_length

    @property
    def start_position(self):
        """CarEnv._load_track: first GRID/STARTLINE segment start (src/car_env.py:235-241)"""
        for s in self.segments:
            if s.segment_type in ("GRID", "STARTLINE"):
                return s.start_position
        return (0.0, 0.0)

    def segment_table(self) -> np.ndarray:
        return np.array([[SEG_TYPES[s.segment_type], s.length, s.start_position[0], s.start_position[1],
                          s.end_position[0], s.end_position[1], s.width, s.curve_angle, s.curve_radius,
                          1.0 if s.curve_direction == "LEFT" else 0.0, s.start_heading, s.end_heading,
                          s.banking_angle] for s in self.segments], np.float64)


def load_track(file_path: str) -> Track:
    """TrackLoader.load_track (src/track_generator.py:305-405)."""
    if not os.path.exists(file_path):
        raise FileNotFoundError(f"Track file not found: {file_path}")
    with open(file_path, "r") as f:
        lines = f.readlines()
    track = Track(name=os.path.splitext(os.path.basename(file_path))[0])
    for line in lines:
        line = line.strip().upper()
        if not line or line.startswith("#"):
            continue
        parts = line.split()
        if not parts:
            continue
        if "#" in line:
            line = line[:line.find("#")].strip()
            parts = line.split()
            if not parts:
                continue
        cmd = parts[0]
        if cmd == "WIDTH":
            if len(parts) != 2:
                raise ValueError(f"WIDTH command requires exactly one argument: {line}")
            try:
                track.width = float(parts[1])
            except ValueError:
                raise ValueError(f"Invalid width value: {parts[1]}")
        elif cmd == "GRID":
            track.add_segment("GRID", DEFAULT_GRID_LENGTH)
        elif cmd == "STARTLINE":
            track.add_segment("STARTLINE", STARTLINE_LENGTH)
        elif cmd == "STRAIGHT":
            if len(parts) < 2 or len(parts) > 3:
                raise ValueError(f"STRAIGHT command requires 1-2 arguments (length [, banking]): {line}")
            # float() raises Python's own "could not convert string to float: 'X'": the reference's re-wrap looks for
            # "invalid literal" (an int() message) and so re-raises float()'s error unchanged (track_generator.py:370-374)
            length = float(parts[1])
            banking = float(parts[2]) if len(parts) == 3 else 0.0
            if banking < -45 or banking > 45:
                raise ValueError(f"Banking angle must be between -45 and 45 degrees: {banking}")
            track.add_segment("STRAIGHT", length, banking_angle=banking)
        elif cmd == "FINISHLINE":
            track.add_segment("FINISHLINE", FINISHLINE_LENGTH)
        elif cmd in ("LEFT", "RIGHT"):
            if len(parts) < 3 or len(parts) > 4:
                raise ValueError(f"{cmd} command requires 2-3 arguments (angle, radius [, banking]): {line}")
            angle, radius = float(parts[1]), float(parts[2])      # float()'s own error, as above (:396-400)
            banking = float(parts[3]) if len(parts) == 4 else 0.0
            if angle <= 0 or angle > 360:
                raise ValueError(f"Curve angle must be between 0 and 360 degrees: {angle}")
            if radius <= 0:
                raise ValueError(f"Curve radius must be positive: {radius}")
            if banking < -45 or banking > 45:
                raise ValueError(f"Banking angle must be between -45 and 45 degrees: {banking}")
            track.add_segment("CURVE", 0, curve_angle=angle, curve_radius=radius, curve_direction=cmd,
                              banking_angle=banking)
        else:
            raise ValueError(f"Unknown command: {cmd}")
    return track


def _wall_from_line(out, x1, y1, x2, y2, thickness):
    """_create_wall_body_from_line (src/car_physics.py:280-339): body def values."""
    cx, cy = (x1 + x2) / 2, (y1 + y2) / 2
    length = ((x2 - x1) ** 2 + (y2 - y1) ** 2) ** 0.5
    if length < 0.1:
        return
    out.append((cx, cy, math.atan2(y2 - y1, x2 - x1), length / 2, thickness / 2))


def build_walls(track: Track) -> np.ndarray:
    """CarPhysics._create_track_walls (src/car_physics.py:118-278) -> [nwall, 5] float64
    (center_x, center_y, angle, half_length, half_thickness) in Box2D creation order."""
    out = []
    for s in track.segments:
        if s.segment_type == "CURVE":
            if s.curve_radius <= 0 or s.curve_angle <= 0:
                continue
            hw = s.width / 2
            shr = math.radians(s.start_heading)
            car = math.radians(s.curve_angle)
            turn = 1.0 if s.curve_direction == "LEFT" else -1.0
            perp = shr + turn * math.pi / 2
            cx = s.start_position[0] + s.curve_radius * math.cos(perp)
            cy = s.start_position[1] + s.curve_radius * math.sin(perp)
            if s.curve_direction == "LEFT":
                ri, ro = s.curve_radius - hw, s.curve_radius + hw
            else:
                ri, ro = s.curve_radius + hw, s.curve_radius - hw
            inner, outer = [], []
            a0 = shr - turn * math.pi / 2
            n = max(PHYSICS_CURVE_MIN_SEGMENTS,
                    min(PHYSICS_CURVE_MAX_SEGMENTS, int(abs(s.curve_angle) / PHYSICS_CURVE_DEGREES_PER_SEGMENT)))
            for i in range(n + 1):
                t = i / n
                ang = a0 + turn * car * t
                if ri > 0:
                    inner.append((cx + ri * math.cos(ang), cy + ri * math.sin(ang)))
                outer.append((cx + ro * math.cos(ang), cy + ro * math.sin(ang)))
            if len(inner) < 2 or len(outer) < 2:
                continue
            for i in range(len(inner) - 1):
                _wall_from_line(out, *inner[i], *inner[i + 1], TRACK_WALL_THICKNESS)
            for i in range(len(outer) - 1):
                _wall_from_line(out, *outer[i], *outer[i + 1], TRACK_WALL_THICKNESS)
        else:
            (sx, sy), (ex, ey) = s.start_position, s.end_position
            hw = s.width / 2
            sl = math.sqrt((ex - sx) ** 2 + (ey - sy) ** 2)
            if sl > 0:
                dx, dy = (ex - sx) / sl, (ey - sy) / sl
                pdx, pdy = -dy, dx
            else:
                pdx, pdy = 0, 1
            _wall_from_line(out, sx + pdx * hw, sy + pdy * hw, ex + pdx * hw, ey + pdy * hw, TRACK_WALL_THICKNESS)
            _wall_from_line(out, sx - pdx * hw, sy - pdy * hw, ex - pdx * hw, ey - pdy * hw, TRACK_WALL_THICKNESS)
    return np.array(out, np.float64).reshape(-1, 5)
