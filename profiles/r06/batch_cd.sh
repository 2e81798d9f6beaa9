#!/bin/bash
# capture / stamps / virtual GPUs (cap_stamps.sh), then the tracer FWD A/B (fwd_ab.sh)
bash profiles/r06/cap_stamps.sh r6c && bash profiles/r06/fwd_ab.sh r6d
