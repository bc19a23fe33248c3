#!/bin/bash
# List the PMC counters rocprofv3 offers on this gfx950 box (TA / TCP / TCC / SQ).
cd /tmp && timeout -k 10 120 rocprofv3 --list-avail > $GRAFT_REPO_ROOT/gpurun_out/pmc_avail.txt 2>&1; echo rc=$?
grep -o "^\s*[A-Z][A-Z0-9_]*" $GRAFT_REPO_ROOT/gpurun_out/pmc_avail.txt | sort -u | tr -d ' ' | grep -E "^(TA_|TCP_|TD_|SQ_WAIT|SQ_INST|SQ_BUSY|SQC_)" | head -150 | tr '\n' ' '
