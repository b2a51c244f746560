"""State-dict (name, shape) lists of the reference modules, in registration order.
TEST INFRASTRUCTURE ONLY (see oracle/reconet_ref.py header).

Order matters: `oracle.seeding.seeded_arrays` walks this list with one generator, exactly as
`gen_golden.py` walked the reference modules' state_dicts.
"""


def _conv(name, cin, cout, k):
    return [(name + ".conv2d.weight", (cout, cin, k, k)), (name + ".conv2d.bias", (cout,))]


def _cir(name, cin, cout, k):
    return _conv(name, cin, cout, k) + [(name + ".instance.weight", (cout,)), (name + ".instance.bias", (cout,))]


def _res(name, c):
    return (_conv(name + ".conv1", c, c, 3) + [(name + ".in1.weight", (c,)), (name + ".in1.bias", (c,))]
            + _conv(name + ".conv2", c, c, 3) + [(name + ".in2.weight", (c,)), (name + ".in2.bias", (c,))])


def reconet(input_frame_num=1):
    """RC/network.py:153-169."""
    s = _cir("conv1", 3 * input_frame_num, 48, 9) + _cir("conv2", 48, 96, 3) + _cir("conv3", 96, 192, 3)
    for i in range(1, 6):
        s += _res(f"res{i}", 192)
    return s + _cir("deconv1", 192, 96, 3) + _cir("deconv2", 96, 48, 3) + _conv("deconv3", 48, 3, 9)


def reconet_sd1(input_frame_num=1):
    """RC/network.py:193-213."""
    s = _cir("conv1", 3 * input_frame_num, 32, 9) + _cir("conv2", 32, 64, 3) + _cir("conv3_sd", 64, 64, 3)
    for i in range(1, 6):
        s += _res(f"res{i}_sd", 64)
    return s + _cir("deconv1_sd", 64, 64, 3) + _cir("deconv2", 64, 32, 3) + _conv("deconv3", 32, 3, 9)


def reconet_sd2(input_frame_num=1):
    """RC/network.py:240-259."""
    s = _cir("conv1_sd2", 3 * input_frame_num, 16, 9) + _cir("conv2_sd2", 16, 32, 3) + _cir("conv3_sd2", 32, 64, 3)
    for i in range(1, 6):
        s += _res(f"res{i}_sd", 64)
    return s + _cir("deconv1_sd2", 64, 32, 3) + _cir("deconv2_sd2", 32, 16, 3) + _conv("deconv3_sd2", 16, 3, 9)


def _vgg(plan_cfg):
    out = []
    cin = 3
    for s, i, cout in plan_cfg:
        out += [(f"slice{s}.{i}.weight", (cout, cin, 3, 3)), (f"slice{s}.{i}.bias", (cout,))]
        cin = cout
    return out


def vgg16():
    """RC/network.py:9-27: torchvision VGG16 features[0:23] as slice1..4."""
    return _vgg([(1, 0, 64), (1, 2, 64), (2, 5, 128), (2, 7, 128), (3, 10, 256), (3, 12, 256), (3, 14, 256),
                 (4, 17, 512), (4, 19, 512), (4, 21, 512)])


def vgg19():
    """AA/vgg19.py:8-41: torchvision VGG19 features[0:30] as slice1..5."""
    return _vgg([(1, 0, 64), (2, 2, 64), (2, 5, 128), (3, 7, 128), (3, 10, 256), (4, 12, 256), (4, 14, 256),
                 (4, 16, 256), (4, 19, 512), (5, 21, 512), (5, 23, 512), (5, 25, 512), (5, 28, 512)])


ADAATTN_LEVELS = ((256, 64 + 128 + 256), (512, 64 + 128 + 256 + 512), (512, 64 + 128 + 256 + 512 + 512))
DECODER = [("conv1", 512, 512, True), ("conv2", 512, 256, True), ("conv3.0", 512, 256, True), ("conv3.1", 256, 256, True),
           ("conv3.2", 256, 256, True), ("conv4", 256, 128, True), ("conv5", 128, 128, True), ("conv6", 128, 64, True),
           ("conv7", 64, 64, True), ("conv8", 64, 3, False)]


def stylizing_network():
    """AA/network.py:223-235 (AdaAttN x3 with 1x1 f/g/h, then Decoder AA/network.py:63-77)."""
    s = []
    for i, (vd, qd) in enumerate(ADAATTN_LEVELS):
        for nm, c in (("f", qd), ("g", qd), ("h", vd)):
            s += [(f"adaattn.{i}.{nm}.weight", (c, c, 1, 1)), (f"adaattn.{i}.{nm}.bias", (c,))]
    for name, cin, cout, relu in DECODER:
        key = f"decoder.{name}.conv.conv" if relu else f"decoder.{name}.conv"
        s += [(key + ".weight", (cout, cin, 3, 3)), (key + ".bias", (cout,))]
    return s


def _rt_conv(name, cin, cout, k):
    return [(name + ".conv.weight", (cout, cin, k, k)), (name + ".conv.bias", (cout,)),
            (name + ".norm.weight", (cout,)), (name + ".norm.bias", (cout,))]


def _rt_deconv(name, cin, cout, k):
    return [(name + ".deconv.weight", (cin, cout, k, k)), (name + ".deconv.bias", (cout,)),
            (name + ".norm.weight", (cout,)), (name + ".norm.bias", (cout,))]


def rtnstv():
    """RT/network.py:65-78 StylizingNetwork."""
    s = _rt_conv("conv1", 3, 16, 3) + _rt_conv("conv2", 16, 32, 3) + _rt_conv("conv3", 32, 48, 3)
    for i in range(1, 6):
        s += _rt_conv(f"res{i}.conv1", 48, 48, 3) + _rt_conv(f"res{i}.conv2", 48, 48, 3)
    return s + _rt_deconv("deconv1", 48, 32, 3) + _rt_deconv("deconv2", 32, 16, 3) + _rt_conv("conv4", 16, 3, 3)


def vgg19_rt():
    """RT/vgg19.py:8-36: torchvision VGG19 features[0:23] as slice1..4 (relu1_2 .. relu4_2)."""
    return _vgg([(1, 0, 64), (1, 2, 64), (2, 5, 128), (2, 7, 128), (3, 10, 256), (3, 12, 256), (4, 14, 256),
                 (4, 16, 256), (4, 19, 512), (4, 21, 512)])
