set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
O=gpurun_out/ktsplit; rm -rf $O; mkdir -p $O
export FA_AB_SHAPES="1,1,256,32,1;1,1,8192,32,1"
CS336_LIB=cs336_systems/_native/variants/base/libcs336_hip.so timeout -k 10 200 rocprofv3 --kernel-trace -d $O/base -o run -- python3 scripts/fa_ab.py > $O/base.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/new -o run -- python3 scripts/fa_ab.py > $O/new.log 2>&1 || exit $?
for v in base new; do echo "== $v"; grep '^{' $O/$v.log; python3 scripts/rocpd_summary.py $O/$v/run_results.db "fa_bwd" | head -20; done
