# drop-in operators (config 2, host edges, C++ mirror) at p = 1 and 8, twice, and the
# isolated host-fold rate. The copy-mode A/B recorded in profiles/r02f_dropin_copy_modes.txt
# ran this with a temporary GS_DIRECT_MAX knob (0: pinned staging for every chunk,
# 262144: this build's split, 2000000: direct copies of every size).
set -e
for rep in 1 2; do
  for p in 1 8; do
    echo "p=$p $(timeout -k 10 120 gelly-streaming_amd/host/bin/dropin_bench 20 0x5EED0020 24 20 $p /tmp/lab.bin | tail -1 | cut -c1-90)"
  done
done
timeout -k 10 200 python tools/host_fold_rate.py | grep -v amdgpu
