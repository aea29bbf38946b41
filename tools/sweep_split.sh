for k in 0 2 4 8; do echo "EKF_CU_SPLIT=$k"; EKF_CU_SPLIT=$k timeout -k 10 200 python tools/kernel_sweep.py || exit 1; done
