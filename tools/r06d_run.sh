bash tools/gpu_ab.sh r06d_xord "base xord0 xord1 xord4 xord16" && bash tools/pmc_req.sh r06d_req "base xord0" "k_pfl_apply"
