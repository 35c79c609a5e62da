#!/bin/bash
# The round's closing GPU check: every -m gpu test, smoke(), and the large-window fuzz on fresh seeds.
SEED0=${SEED0:-99500} bash "$(dirname "$0")/session.sh" ${TAG:-r6zx} pytest smoke fuzz_large
