set -e
for i in 1 2; do
timeout -k 10 120 python bench.py --cpu-sample 0 --steps 10 > gpurun_out/b_t.json 2>/dev/null; python -c "import json;d=json.load(open('gpurun_out/b_t.json'));print('timing',d['ms_per_step'])"
timeout -k 10 120 python bench.py --cpu-sample 0 --steps 10 --no-timing > gpurun_out/b_nt.json 2>/dev/null; python -c "import json;d=json.load(open('gpurun_out/b_nt.json'));print('notiming',d['ms_per_step'])"
KARMA_OVERLAP=1 timeout -k 10 120 python bench.py --cpu-sample 0 --steps 10 --no-timing > gpurun_out/b_ov.json 2>/dev/null; python -c "import json;d=json.load(open('gpurun_out/b_ov.json'));print('overlap notiming',d['ms_per_step'])"
done
