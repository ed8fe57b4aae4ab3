set -e
L=quickcheck-state-machine-distributed_amd/lib
for i in 1 2 3; do
for lib in libqsmd.so libqsmd_bf.so; do
  timeout -k 10 120 python tools/ab_lib.py $L/$lib bank_4x16 2>/dev/null
done
done
