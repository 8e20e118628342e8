#!/bin/bash
# round-3 final: GPU suite + smoke + driver-shaped bench, then the rocprofv3 step breakdown of the bench window
set -o pipefail
bash tools/gpurun/suite_bench.sh || exit 1
bash tools/gpurun/archive/r3_steps.sh || exit 1
