#!/bin/bash
# run the ablation bench with an environment switch:  tools/abl_env.sh NAME VAR=VALUE ...
name="$1"; shift
env "$@" python tools/ablate.py run "$name"
