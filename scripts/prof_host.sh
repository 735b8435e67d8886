mkdir -p gpurun_out && timeout -k 10 300 python -c "
import cProfile, pstats, sys
sys.argv = ['bench.py', '--steps', '300', '--warmup', '5', '--series', '12500']
import runpy
cProfile.run('runpy.run_path(\"bench.py\", run_name=\"__main__\")', 'gpurun_out/host.prof')
p = pstats.Stats('gpurun_out/host.prof'); p.sort_stats('tottime').print_stats(30)
" > gpurun_out/host_prof.txt 2>&1
