# round 2: HIP graph replay of the native batch loop vs stream launches (config B, emit)
bash tools/gpu_session.sh \
 "g60:200:python tools/graph_probe.py 60 4" \
 "g198:200:python tools/graph_probe.py 198 2" \
 "g6:200:python tools/graph_probe.py 6 40"
