#!/bin/bash
# s_setprio(2) for the raw path's general-range waves (full chunks): ramp A/B
set -o pipefail
VARS="ramp rand" bash tools/ab_lib.sh gprio_c5
