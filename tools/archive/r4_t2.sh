#!/bin/bash
# tiled route: tests + webbase/cant lines, then kernel stats of the webbase tiled leg
set -uo pipefail
TAG=${1:-r4t}
bash tools/r4_tiled.sh $TAG && bash tools/r4_ks.sh ${TAG}_ks --matrix webbase --leg tiled
