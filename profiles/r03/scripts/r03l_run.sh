# round 3: occupancy sensitivity of the render (LDS padding per block: 32 / 24 / 20 / 16 waves per CU)
set -o pipefail
bash tools/ab_libs.sh occ base occ24 occ20 occ16 > gpurun_out/r03l_occ.txt 2>&1
