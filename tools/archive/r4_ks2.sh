#!/bin/bash
# kernel stats of the webbase device pass and the webbase tiled leg
set -uo pipefail
TAG=${1:-r4k}
bash tools/r4_ks.sh ${TAG}_dev --matrix webbase && bash tools/r4_ks.sh ${TAG}_tiled --matrix webbase --leg tiled
