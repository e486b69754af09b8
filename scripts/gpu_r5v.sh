#!/bin/bash
# r5u (final-partition A/B) then r5t (histogram issue / wait counters)
set -o pipefail
./scripts/gpu_r5u.sh && ./scripts/gpu_r5t.sh
