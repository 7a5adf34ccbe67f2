import os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from nascargymnasium_amd.batched import BatchedCarEnv
from nascargymnasium_amd.track import track_path
for t in sorted(f[:-6] for f in os.listdir("nascargymnasium_amd/tracks") if f.endswith(".track")):
    print(t, flush=True); e = BatchedCarEnv(1, 1, track_path(t), device="cuda:0"); e.close()
