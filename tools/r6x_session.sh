#!/bin/bash
# Round-4 session X (final tree): C2 per-sample line, C3 and C5 lines (C5 with its per-sample leg).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
C5PS=1 bash tools/gpu_session.sh R6x c2ps c3b c5b
