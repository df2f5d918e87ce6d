set -u
O=gpurun_out/r03c; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/conv_lab.py abconv --lib ab/librrin_hip_prev.so --lib-b rrin_amd/librrin_hip.so,ab/librrin_hip_ilp.so,ab/librrin_hip_nofence.so --batch 2 --reps 10 --rounds 5 --shapes 256:256:3:1:18,64:32:0:1:18,32:32:0:1:18,128:64:1:1:18,512:512:4:1:18,32:32:0:2:18,512:1024:4:4:18 > $O/ab.log 2>&1; echo rc=$?; grep -v amdgpu.ids $O/ab.log
