cd $GRAFT_REPO_ROOT; O=gpurun_out/${1:-r11e}; mkdir -p $O
PUCFEM_PROJ_SPMV=1 timeout -k 10 200 python -u tools/pcg_trace.py 7 1e-12 40 0 > $O/trace_tight_spmv.txt 2>&1 &&
PUCFEM_PROJ_SPMV=1 timeout -k 10 200 python -u tools/pcg_trace.py 7 5e-8 116 104 > $O/trace_spmv.txt 2>&1
