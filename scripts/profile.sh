# rocprofv3 evidence for the bench kernel: kernel trace + stats, then one PMC
# counter per pass (FETCH_SIZE, WRITE_SIZE) -- never combined with other traces.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/prof
TAG=${TAG:-r03}
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace -o $TAG --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu --timed-only > gpurun_out/prof/trace.log 2>&1 && \
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/fetch -o ${TAG}_fetch --output-format csv -- python3 bench.py --steps 3 --warmup 0 --no-cpu --timed-only > gpurun_out/prof/fetch.log 2>&1 && \
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof/write -o ${TAG}_write --output-format csv -- python3 bench.py --steps 3 --warmup 0 --no-cpu --timed-only > gpurun_out/prof/write.log 2>&1
rc=$?; echo "profile rc=$rc"; tail -2 gpurun_out/prof/trace.log; find gpurun_out/prof -name "*.csv" | sort; exit $rc
