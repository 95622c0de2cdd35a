set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_session.sh r02d || exit $?
timeout -k 10 300 python tools/time_pytree.py > gpurun_out/r02d_pytree.json 2>gpurun_out/r02d_pytree.err || exit $?
cat gpurun_out/r02d_pytree.json
