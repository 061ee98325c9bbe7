set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/fl_profile.py > gpurun_out/r04ad_fl_profile.txt 2> gpurun_out/r04ad_fl_profile.err || { tail -20 gpurun_out/r04ad_fl_profile.err; exit 2; }
echo ok
