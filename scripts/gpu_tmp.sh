bash scripts/gpu_lap2.sh > gpurun_out/lap2.out 2>&1; rc=$?; tail -3 gpurun_out/lap2.out; [ $rc -eq 0 ] || exit $rc
LIBS="pd2 pd3 pd6" SPECS="64:TSA_LAP_M=1,TSA_LAP_NW=4 64:TSA_LAP_M=1,TSA_LAP_NW=8 128:TSA_LAP_M=1,TSA_LAP_NW=4 256:TSA_LAP_M=1,TSA_LAP_NW=4 256:TSA_LAP_M=1,TSA_LAP_NW=8 512:TSA_LAP_M=1,TSA_LAP_NW=4" bash scripts/gpu_lapvar.sh
