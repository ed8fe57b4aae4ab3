set -e
L=quickcheck-state-machine-distributed_amd/lib
for i in 1 2; do
for lib in libqsmd.so libqsmd_t5.so; do
  timeout -k 10 120 python tools/ab_lib.py $L/$lib ticket_2x10 2>/dev/null
done
done
