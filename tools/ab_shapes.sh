export TMPDIR=/tmp; mkdir -p gpurun_out/ab
timeout -k 10 300 python tools/ab_libs.py c3 6 mjpeg423-video-decoder-software_amd/libmj423gpu.so tools/variants/b420_16x128/libmj423gpu.so > gpurun_out/ab/c3.log 2>&1 || { tail -20 gpurun_out/ab/c3.log; exit 1; }
cat gpurun_out/ab/c3.log
timeout -k 10 300 python tools/ab_libs.py c2 6 mjpeg423-video-decoder-software_amd/libmj423gpu.so tools/variants/b420_16x128/libmj423gpu.so > gpurun_out/ab/c2.log 2>&1 || { tail -20 gpurun_out/ab/c2.log; exit 1; }
cat gpurun_out/ab/c2.log
timeout -k 10 300 python tools/ab_libs.py c5 6 mjpeg423-video-decoder-software_amd/libmj423gpu.so tools/variants/b422_32x128/libmj423gpu.so > gpurun_out/ab/c5.log 2>&1 || { tail -20 gpurun_out/ab/c5.log; exit 1; }
cat gpurun_out/ab/c5.log
