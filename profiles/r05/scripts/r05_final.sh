#!/bin/bash
# Round-5 HEAD check: the whole GPU suite, smoke, the default bench line, then the C2 profiles
# (rocprofv3 stats + PMC passes, scripts/r05_prof.sh).
set -o pipefail
bash scripts/r05_full.sh ${1:-final} || exit $?
bash scripts/r05_prof.sh || exit $?
