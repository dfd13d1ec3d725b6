# round 4: host-side profile of the eager config-3 union step (tools/host_profile_union.py)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/host_profile_union.py --steps 10 > gpurun_out/host_prof.txt 2> gpurun_out/host_prof.err || { tail -30 gpurun_out/host_prof.err; exit 1; }
head -1 gpurun_out/host_prof.txt
timeout -k 10 300 python -u tools/host_profile_union.py --steps 10 --same-thread --top 70 --callers "parameters|named_modules|_named_members" > gpurun_out/host_prof_st.txt 2> gpurun_out/host_prof_st.err || { tail -30 gpurun_out/host_prof_st.err; exit 1; }
head -1 gpurun_out/host_prof_st.txt
