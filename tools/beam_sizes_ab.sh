#!/bin/bash
# beam-list sizes per library variant (NASCAR_VERBOSE build log of nascar_add_track), all 8 tracks
cd "$GRAFT_REPO_ROOT" || exit 1
for L in "$@"; do
  echo "== $L"
  NASCAR_LIB="$GRAFT_REPO_ROOT/$L" timeout -k 10 120 python tools/beam_sizes.py 2>&1 | grep "beam grid" | sed 's/nascar_add_track: //'
done
