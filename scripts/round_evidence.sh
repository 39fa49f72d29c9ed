#!/bin/bash
# The round's evidence in one GPU call: scripts/round_profile.sh (GPU tests,
# smoke, the default bench line, its kernel stats, FETCH / WRITE PMC passes),
# then the C4 / C5 lines and the emulated rank-of-N steps (scale_probe.sh).
set -u
bash scripts/round_profile.sh || exit $?
bash scripts/scale_probe.sh || exit $?
