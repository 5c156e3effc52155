SE3ICP_LIB=$PWD/se3-icp_amd/lib_prof/libse3icp.so timeout -k 10 200 python bench.py --steps 1 --warmup 0 --cpu-baseline off --secondary off > gpurun_out/prof_new.json 2> gpurun_out/prof_new.err
