#!/bin/bash
# Same-process A/B of a per-minibatch update switch (tools/kbench.py update_env; KB_VAR / KB_VALUES).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
KB_ROUNDS=${KB_ROUNDS:-15} timeout -k 10 240 python tools/kbench.py update_env
