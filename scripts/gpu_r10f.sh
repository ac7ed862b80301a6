set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=24
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/nprof_r10f -o run -- python3 tools/normals_prof.py 8 > gpurun_out/r10f_normals.log 2>&1 || exit 1
grep -i "normals" $(find gpurun_out/nprof_r10f -name "*kernel_stats.csv") | cut -c1-60,100-180
RST_KNN_GRID=0 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/nprof0_r10f -o run -- python3 tools/normals_prof.py 8 > gpurun_out/r10f_normals0.log 2>&1 || exit 1
grep -i "normals" $(find gpurun_out/nprof0_r10f -name "*kernel_stats.csv") | cut -c1-60,100-180
for pt in 3 1; do
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --prep-threads $pt --no-cpu --no-host-api --no-gicp > gpurun_out/r10f_bench_pt$pt.log 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/r10f_bench_pt$pt.log').read().strip().splitlines()[-1]);print('prep threads $pt value', round(d['value']), 'fp64', round(d['fp64_sums']['iterations_per_s']), 'p2plane', round(d['p2plane']['iterations_per_s']), round(d['p2plane']['frames_per_s']), 'knn', round(d['p2plane']['knn16_normals']['iterations_per_s']), round(d['p2plane']['knn16_normals']['frames_per_s']))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/shard_r10f -o run -- python3 bench.py --workload sharded --steps 3 --warmup 1 --no-cpu > gpurun_out/r10f_sharded.log 2>&1 || exit 1
python3 scripts/iter_profile_all.py $(find gpurun_out/shard_r10f -name "*kernel_trace.csv") > gpurun_out/r10f_sharded_iteration_profile.txt
tail -3 gpurun_out/r10f_sharded_iteration_profile.txt | cut -c1-600
timeout -k 10 300 python bench.py --workload pyramid --graphs --no-p2plane --steps 96 > gpurun_out/r10f_pyramid.log 2>&1 || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/r10f_pyramid.log').read().strip().splitlines()[-1]);print('pyramid', round(d['value']), round(d['frames_per_s'],1), d['roofline']['frac'])"
