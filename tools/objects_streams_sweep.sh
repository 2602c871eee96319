cd "${GRAFT_REPO_ROOT:-/root/repo}"
for T in 2 3 4 8 2 3; do
  timeout -k 10 300 python bench.py --frames 8 --steps 1 --cpu-frames 0 --filter-frames 0 --hybrid-objects 0 \
      --object-streams $T > gpurun_out/b_obj_$T.log 2>&1 || { tail -20 gpurun_out/b_obj_$T.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/b_obj_$T.log') if l.startswith('{')][-1]); o=d['objects']; print('streams $T', o['ms'], o['frames_per_s'], o['merged_points'])"
done
