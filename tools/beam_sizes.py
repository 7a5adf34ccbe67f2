"""Print the beam-list / head sizes of every bundled track (NASCAR_VERBOSE build log of nascar_add_track)."""
import os
import sys
os.environ["NASCAR_VERBOSE"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nascargymnasium_amd.batched import BatchedCarEnv  # noqa: E402
from nascargymnasium_amd.track import available_tracks  # noqa: E402
BatchedCarEnv(8, 1, available_tracks(), device="cuda:0").close()
