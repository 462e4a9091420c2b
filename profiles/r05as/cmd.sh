TAG=r05as bash tools/gpu_prof.sh
