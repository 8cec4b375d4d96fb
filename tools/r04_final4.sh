#!/bin/bash
# Round-4 final tree (placed hop tables): the round profile of the headline (bench with the
# CPU baseline and the vendor comparator, kernel stats, FETCH/WRITE/L2 PMC passes).
set -euo pipefail
bash tools/profile_round.sh r04final3
echo done
