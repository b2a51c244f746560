"""Algorithmic FLOPs of one ReCoNet training step (reference semantics) per frame pair."""
H, W = 256, 512


def conv(cin, cout, k, h, w):
    return 2.0 * cin * cout * k * k * h * w


def reconet_fwd(H, W):
    L = [conv(3, 48, 9, H, W), conv(48, 96, 3, H // 2, W // 2), conv(96, 192, 3, H // 4, W // 4)]
    L += [conv(192, 192, 3, H // 4, W // 4)] * 10
    L += [conv(192, 96, 3, H // 2, W // 2), conv(96, 48, 3, H, W), conv(48, 3, 9, H, W)]
    return L


def vgg16(H, W):
    cfg = [(3, 64, 1), (64, 64, 1), (64, 128, 2), (128, 128, 2), (128, 256, 4), (256, 256, 4), (256, 256, 4),
           (256, 512, 8), (512, 512, 8), (512, 512, 8)]
    return [conv(a, b, 3, H // s, W // s) for a, b, s in cfg]


def gram(H, W):
    return [2.0 * c * c * (H // s) * (W // s) for c, s in ((64, 1), (128, 2), (256, 4), (512, 8))]


if __name__ == "__main__":
    rf = reconet_fwd(H, W)
    v = vgg16(H, W)
    g = gram(H, W)
    per_pair = {
        "stylizer fwd (2 frames)": 2 * sum(rf),
        "stylizer dgrad (no conv1)": 2 * sum(rf[1:]),
        "stylizer wgrad": 2 * sum(rf),
        "vgg16 fwd (4 images)": 4 * sum(v),
        "vgg16 dgrad (2 styled)": 2 * sum(v),
        "gram fwd+bwd (2 styled)": 2 * 3 * sum(g),
    }
    tot = sum(per_pair.values())
    for k, x in per_pair.items():
        print(f"{k:28s} {x/1e9:8.1f} GF")
    print(f"{'total per pair':28s} {tot/1e9:8.1f} GF   (B=8: {8*tot/1e12:.2f} TF/step)")
    print(f"vgg19 features[0:21] fwd per frame: see BASELINE (63.27 GF); vgg16 fwd per frame {sum(v)/1e9:.2f} GF")
