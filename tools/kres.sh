# per-kernel VGPR / AGPR / scratch / LDS of one HIP source (host-side compile only)
f=$1
cd /tmp && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c "$f" -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage 2>&1 \
 | grep -E "error|Function Name|VGPRs:|AGPRs:|ScratchSize|LDS Size" \
 | sed -E 's/.*remark: *//; s/ \[-Rpass.*//; s/_ZN5gasfm12_GLOBAL__N_1[0-9]+//; s/EEEv.*//' | paste -sd' ' | sed 's/Function Name: /\n/g'
echo
