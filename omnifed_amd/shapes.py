"""Named-parameter shapes of the benchmark configurations (BASELINE.json ``configs``).

Weights are never loaded (no network, no checkpoints): only ``named_parameters()``
order and shapes matter to the codec.

* ``resnet18``  — torchvision ResNet-18, CIFAR-10 head (10 classes): 62 tensors,
  11 181 642 elements (``conf/test_fedavg_centralized_torchdist_cifar10_resnet18.yaml:31-32``).
* ``llama150m`` — LlamaConfig(vocab 32000, hidden 1024, intermediate 2688, 12 layers,
  untied head): 111 tensors, 214 983 680 elements.
* ``llama400m`` — same with intermediate 4096, 20 layers: 183 tensors, 401 122 304 elements.
"""

from __future__ import annotations

from typing import List, Tuple

Shape = Tuple[int, ...]


def resnet18(num_classes: int = 10) -> List[Tuple[str, Shape]]:
    out: List[Tuple[str, Shape]] = [("conv1.weight", (64, 3, 7, 7)), ("bn1.weight", (64,)), ("bn1.bias", (64,))]
    cin = 64
    for li, cout in enumerate((64, 128, 256, 512), start=1):
        for b in range(2):
            p = f"layer{li}.{b}"
            c_in = cin if b == 0 else cout
            out += [(f"{p}.conv1.weight", (cout, c_in, 3, 3)), (f"{p}.bn1.weight", (cout,)), (f"{p}.bn1.bias", (cout,)),
                    (f"{p}.conv2.weight", (cout, cout, 3, 3)), (f"{p}.bn2.weight", (cout,)), (f"{p}.bn2.bias", (cout,))]
            if b == 0 and li > 1:
                out += [(f"{p}.downsample.0.weight", (cout, cin, 1, 1)), (f"{p}.downsample.1.weight", (cout,)),
                        (f"{p}.downsample.1.bias", (cout,))]
        cin = cout
    out += [("fc.weight", (num_classes, 512)), ("fc.bias", (num_classes,))]
    return out


def llama(vocab: int, hidden: int, inter: int, layers: int) -> List[Tuple[str, Shape]]:
    out: List[Tuple[str, Shape]] = [("model.embed_tokens.weight", (vocab, hidden))]
    for i in range(layers):
        p = f"model.layers.{i}"
        out += [(f"{p}.self_attn.q_proj.weight", (hidden, hidden)), (f"{p}.self_attn.k_proj.weight", (hidden, hidden)),
                (f"{p}.self_attn.v_proj.weight", (hidden, hidden)), (f"{p}.self_attn.o_proj.weight", (hidden, hidden)),
                (f"{p}.mlp.gate_proj.weight", (inter, hidden)), (f"{p}.mlp.up_proj.weight", (inter, hidden)),
                (f"{p}.mlp.down_proj.weight", (hidden, inter)), (f"{p}.input_layernorm.weight", (hidden,)),
                (f"{p}.post_attention_layernorm.weight", (hidden,))]
    out += [("model.norm.weight", (hidden,)), ("lm_head.weight", (vocab, hidden))]
    return out


CONFIGS = {
    "resnet18": lambda: resnet18(10),
    "llama150m": lambda: llama(32000, 1024, 2688, 12),
    "llama400m": lambda: llama(32000, 1024, 4096, 20),
}


def numel(shape: Shape) -> int:
    n = 1
    for d in shape:
        n *= int(d)
    return n


def model_shapes(name: str) -> List[Tuple[str, Shape]]:
    if name not in CONFIGS:
        raise ValueError(f"unknown config {name!r}; expected one of {sorted(CONFIGS)}")
    return CONFIGS[name]()
