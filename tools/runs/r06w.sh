set -e
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/datacos_plugin.py --algo earlyfusion --frames 240 --beat-period 5 --tracks 15000 --out gpurun_out/r06w_datacos_earlyfusion_15000.json > gpurun_out/r06w_datacos_earlyfusion_15000.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r06w_ef -o run -- python3 -u tools/datacos_plugin.py --algo earlyfusion --frames 240 --beat-period 5 --tracks 15000 --sample 200 --host-eval-keys , --out gpurun_out/r06w_ef_prof.json > gpurun_out/r06w_ef_prof.txt 2>&1
