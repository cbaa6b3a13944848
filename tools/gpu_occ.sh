mkdir -p gpurun_out && timeout -k 10 240 ./tools/microbench/layout_bw > gpurun_out/layout_bw_r02z.txt 2>&1; tail -6 gpurun_out/layout_bw_r02z.txt
A=EVAM_PP_LIB=$PWD/ab/libevam_pp_sgpr80.so; B=EVAM_PP_LIB=$PWD/ab/libevam_pp_sgpr96.so
bash tools/sweep_env.sh occ c2 "EVAM_PP_ABLATE=0|$A|$B|EVAM_PP_ABLATE=0|$A|$B" && bash tools/sweep_env.sh occ c5 "EVAM_PP_ABLATE=0|$A|EVAM_PP_ABLATE=0|$A" && bash tools/sweep_env.sh occ c4 "EVAM_PP_ABLATE=0|$A|EVAM_PP_ABLATE=0|$A"
