"""Test-time render graph sizes (renderer.TestRenderer iters_per_graph / iters_tail) on ONE trained state:
trains the bench's Lego-shaped scene for --pretrain steps, then renders the same 20 frames with each
configuration, alternating, --reps times (bench.inference_bench: frames per second and ms per frame per
sample/ray; every configuration's pixels equal the host loop's bit for bit).  Diagnostics (GPU box)."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ar-nerf_amd")]

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pretrain", type=int, default=2000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--configs", default="16:8,24:4,32:4,28:2")
    a = ap.parse_args()
    import synthetic as S
    from trainer import NGPTrainer
    torch.cuda.set_device(0)
    scene = S.AnalyticScene(W=800, H=800, n_images=100, scale=0.5)
    tr = NGPTrainer(scale=0.5, batch_size=8192, device="cuda")
    gt = scene.gt_images(device="cuda")
    dirs, poses = scene.directions.cuda().contiguous(), scene.poses.cuda().contiguous()
    t0 = time.time()
    for _ in range(a.pretrain):
        tr.train_step(gt, dirs, poses)
    tr.drain()
    torch.cuda.synchronize()
    print(f"pretrain {a.pretrain} steps {time.time() - t0:.1f}s", flush=True)
    cfgs = [tuple(int(v) for v in c.split(":")) for c in a.configs.split(",")]
    for rep in range(a.reps):
        for k, t in cfgs:
            out = bench.inference_bench(tr, 800, 20, 1, 0, iters_per_graph=k, iters_tail=t)
            print(f"rep {rep} graphs {k}/{t}: fps {out['fps']}, ms/frame {out['ms_per_frame']}, iterations "
                  f"{out['iterations_per_frame']}, samples/ray {out['samples_per_ray']}, ms per sample/ray "
                  f"{out['ms_per_frame_per_sample_per_ray']}, bit-exact {out['host_loop_bit_exact']}", flush=True)


if __name__ == "__main__":
    main()
