# round 2: pinned H2D rate over 1 / 2 / 3 streams, with and without a concurrent D2H
bash tools/gpu_session.sh \
 "h2d:200:python tools/h2d_probe.py 256" \
 "h2d64:200:python tools/h2d_probe.py 64"
