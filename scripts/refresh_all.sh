#!/bin/bash
# profiles/r01 refresh (single engine: kernel stats, PMC bytes, SQ counters, phase stamps) and the group profile
set -o pipefail
bash scripts/refresh_profiles.sh || exit 1
bash scripts/profile_group.sh || exit 2
