#!/bin/bash
bash profiles/r06/cap_diag.sh r6e; bash profiles/r06/fwd_ab.sh r6d
