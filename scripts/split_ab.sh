set -u
timeout -k 10 300 python -u scripts/envs_ab.py 1000 8 nosplit=RT_TAIL_TILES_PM:1000 default=RT_TAIL_TILES_PM:- > gpurun_out/ab_split.log 2>&1 || exit 1
timeout -k 10 400 python -u scripts/envs_ab.py 10000 6 nosplit=RT_TAIL_TILES_PM:1000 default=RT_TAIL_TILES_PM:- >> gpurun_out/ab_split.log 2>&1 || exit 1
AB_W=3840 AB_H=2160 AB_K=158 timeout -k 10 300 python -u scripts/envs_ab.py 1000 6 nosplit=RT_TAIL_TILES_PM:1000 default=RT_TAIL_TILES_PM:- tail3=RT_SAMPLE_CHUNKS:3 >> gpurun_out/ab_split.log 2>&1 || exit 1
timeout -k 10 200 python -u scripts/rows_map_ab.py 1000 hash >> gpurun_out/ab_split.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/ab_split.log; exit $rc
