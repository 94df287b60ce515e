#!/bin/bash
# C3 A/B of the asynchronous pass tail (tail_async 0 vs the default 1)
set -u
bash tools/c3_opts.sh "tail_async=0" "" "tail_async=0" ""
