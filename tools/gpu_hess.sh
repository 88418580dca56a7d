#!/bin/bash
# exact-Hessian interior point: GPU Hessian vs oracle, then the IP GPU tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/gpu_hess_check.py ip_go2_rnea_n20_stand ip_go2_cv_n20_stand ip_go2_cv_nb_n20 ip_go2_ca_n20 ip_go2_acc_nb_n20 ip_b2g_rnea_n50 ip_b2g_acc_n50 ip_b2_aba_n40 > gpurun_out/hess_check.log 2>&1
