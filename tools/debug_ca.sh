R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
for cfg in "32 1 20 128" "32 1 2 128" "8 1 3 0" "32 2 3 0"; do
  set -- $cfg; t="$1_$2_$3_$4"
  timeout -k 10 120 python tools/debug_ca.py new_$t $cfg > /dev/null 2>>gpurun_out/dbg.err || exit 1
  SRMI_LIB=$R/alt/libsrmi_prev.so timeout -k 10 120 python tools/debug_ca.py old_$t $cfg > /dev/null 2>>gpurun_out/dbg.err || exit 2
  python -c "
import torch; a=torch.load('gpurun_out/dbg_new_$t.pt'); b=torch.load('gpurun_out/dbg_old_$t.pt')
d=(a-b).double(); print('$cfg', float(d.norm()/b.double().norm()), 'bad tiles', [i for i in range(a.shape[0]) if float(d[i].norm()/b[i].double().norm())>1e-2])"
done
