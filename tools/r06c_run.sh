bash tools/r04_final.sh r06c && bash tools/r06_ab_cfg.sh r06c_ab "base bytew" "c1,c2zipf" && bash tools/gpu_ab.sh r06c_lr "base laterank"
