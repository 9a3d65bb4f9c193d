#!/bin/bash
# tools/knob_ab.sh on the LOKI workload (PAGED)
BENCH_ARGS="--workload loki ${BENCH_ARGS}" exec bash "$(dirname "$0")/knob_ab.sh" "$@"
