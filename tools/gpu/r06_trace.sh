# round 6: kernel trace of exactly the bench's timed C2 step (three decoder streams) and the
# wall-time account per kernel class (tools/trace_step.py + tools/schedule_account.py)
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
O=gpurun_out/r06_trace; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/tr -o run -- python3 tools/trace_step.py --steps 2 > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
K=$(ls $O/tr/*kernel_trace.csv | head -1)
python3 tools/schedule_account.py $K --steps 2 > $O/account.txt 2>&1 || { tail -5 $O/account.txt; exit 1; }
rm -rf $O/tr
cat $O/account.txt
