# Round 6: the vector-memory pipeline counters of the C3-regime workloads on the closing build
# (tools/vmem_study.sh; reduced by tools/c2_study.py into profiles/r06_experiments/vmem_pipeline.json)
cd /root/repo
bash tools/vmem_study.sh vmem6_air "--scene airplane_knot --spp 64" "product|" && \
bash tools/vmem_study.sh vmem6_knot "--scene torusknot --spp 64" "product|"
