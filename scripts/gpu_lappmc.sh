#!/bin/bash
# SQ counters of single-cube lap launches (two passes, 8 SQ counters each),
# over tools/lap_trace.py specs (default: one unchained workgroup, NW = 4).
set -o pipefail
R="$GRAFT_REPO_ROOT"; TAG=${TAG:-lapsq}
cd /tmp && export TMPDIR=/tmp
export TSA_PKG_DIR=${TSA_PKG_DIR:-$GRAFT_REPO_ROOT/variants/diag}  # TSA_LAP_SINGLE needs the -DTSA_DIAG build
OUT="$R/gpurun_out/pmc_${TAG}"; mkdir -p "$OUT"
S=${SPECS:-"64x8x64:TSA_LAP_M=1,TSA_LAP_NW=4,TSA_LAP_SINGLE=1"}
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace -d "$OUT/p$i" -o run --output-format csv \
    -- python3 "$R/tools/lap_trace.py" --reps 2 $S > "$OUT/p$i.json" 2> "$OUT/p$i.err"
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/p$i.err"; exit $rc; }
done
find "$OUT" -name "*counter_collection.csv" | head
