#!/bin/bash
# A/B of library variants on the LiveJournal row blocks (heaviest + a 60,000-row block):
#   bash tools/ljab.sh TAG "variant ..."
set -uo pipefail
TAG=$1; VARS=$2
bash tools/ab.sh ${TAG}_ljh "$VARS" --matrix lj --row-start 1883808 --rows 1600 || exit 1
bash tools/ab.sh ${TAG}_ljm "$VARS" --matrix lj --row-start 2000000 --rows 60000 --steps 3 || exit 1
