# ingress A/B rehearsal (CPU echo, 8 ranks + 2-rank real-engine protocol) then round-3 PMC passes
bash tools/gpu_ingress2.sh > gpurun_out/ingress_summary.txt 2>&1 || exit $?
bash tools/gpu_pmc_r3.sh
