"""Print the beam-list / head sizes of every bundled track (NASCAR_VERBOSE build log of nascar_add_track)."""
import os
os.environ["NASCAR_VERBOSE"] = "1"
from nascargymnasium_amd.batched import BatchedCarEnv  # noqa: E402
from nascargymnasium_amd.track import available_tracks  # noqa: E402
BatchedCarEnv(8, 1, available_tracks(), device="cuda:0").close()
