#!/bin/bash
# GPU box: TLB and memory-side stall counters of the batch kernel on six buffer pairs
# (tools/probe PROBE_PAIRS), to find what makes one allocation faster than another.
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r02pp; mkdir -p $O
P=$GRAFT_REPO_ROOT/tools/probe
cd $GRAFT_REPO_ROOT
PROBE_PAIRS=6 timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS TCP_UTCL1_TRANSLATION_HIT TCP_UTCL1_STALL_MULTI_MISS TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS -d $O/t1 -o p --output-format csv -- $P 420 3840 2160 300 3 > $O/t1.log 2>&1 || { tail -5 $O/t1.log; exit 1; }
PROBE_PAIRS=6 timeout -s KILL 120 rocprofv3 --pmc TCC_TAG_STALL TCC_EA0_WRREQ_STALL TCC_TOO_MANY_EA_WRREQS_STALL TCC_EA0_RDREQ_DRAM_CREDIT_STALL -d $O/t2 -o p --output-format csv -- $P 420 3840 2160 300 3 > $O/t2.log 2>&1 || { tail -5 $O/t2.log; exit 1; }
PROBE_PAIRS=6 timeout -s KILL 120 rocprofv3 --pmc TA_ADDR_STALLED_BY_TC_CYCLES TA_DATA_STALLED_BY_TC_CYCLES GRBM_GUI_ACTIVE -d $O/t3 -o p --output-format csv -- $P 420 3840 2160 300 3 > $O/t3.log 2>&1 || { tail -5 $O/t3.log; exit 1; }
grep pair $O/t1.log $O/t2.log $O/t3.log
echo pp done
