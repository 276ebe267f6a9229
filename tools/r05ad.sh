#!/bin/bash
# stereo tile size (C3, C5) and persistent FIR grid (C5) A/B
bash tools/ab_env.sh r05ad "base||base" "st2k||st2k" "st8k||st8k" "base2||base" "st2kb||st2k" "st8kb||st8k" || exit $?
bash tools/ab_cfg.sh r05ad C5 6 "base||base" "st2k||st2k" "st8k||st8k" "cus192|MSGPU_FIR8P_CUS=192|base" "cus224|MSGPU_FIR8P_CUS=224|base" "base2||base"
