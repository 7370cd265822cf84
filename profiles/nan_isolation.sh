# Round-2 isolation of the round-1 pixel-bandwidth NaN, recipe as run:
# two trees of commit f6c18db (which introduced PixbwTrainStep together with the overflow-robust
# compositing), "nofix" with den_render.hip / den_device.h of its parent, both with the synthetic
# camera speed set back to 0.5 units/s; each runs the pixel-bandwidth bench for 6 steps.
# Result: profiles/r02_nan_isolation.txt.
set -e
rm -rf _naniso && mkdir -p _naniso/fix _naniso/nofix
for t in fix nofix; do git archive f6c18db | tar -x -C _naniso/$t; done
git show f6c18db^:deblur-e-nerf_amd/csrc/den_render.hip > _naniso/nofix/deblur-e-nerf_amd/csrc/den_render.hip
git show f6c18db^:deblur-e-nerf_amd/csrc/den_device.h > _naniso/nofix/deblur-e-nerf_amd/csrc/den_device.h
for t in fix nofix; do
  sed -i 's/seed=1234, rank=0, world=1, speed=5.0)/seed=1234, rank=0, world=1, speed=0.5)/' \
    _naniso/$t/deblur-e-nerf_amd/deblur_e_nerf/train.py
  make -s -C _naniso/$t/deblur-e-nerf_amd/csrc
done
# on the GPU box:
#   for t in nofix fix; do (cd _naniso/$t && timeout -k 10 300 python bench.py --pixbw --steps 6 --warmup 0 \
#     --no-cpu-baseline > ../../gpurun_out/nan_$t.log 2>&1) || break; done
