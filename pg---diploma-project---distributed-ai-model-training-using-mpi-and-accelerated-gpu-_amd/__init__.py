"""pgdist — MI355X-native data-parallel image-classification training framework.

Capabilities mirror the reference project (MobileNetV2 fine-tuning on CIFAR-10
at 224x224 with serial / single-GPU / MPI+DDP modes, best-model checkpoint,
top-k inference and a web demo), re-designed for AMD Instinct
MI355X (gfx950):

* ``pgdist.models``   — MobileNetV2 / ResNet-50 with torchvision-compatible
  ``state_dict`` keys (reference: ``cifar10_serial_mobilenet_224.py:70-73``).
* ``pgdist.ops``      — hand-written HIP/CDNA4 kernels (NHWC bf16 depthwise and
  MFMA pointwise convolutions with fused BatchNorm/ReLU6, fused head + CE,
  fused Adam, GPU augmentation) loaded from the in-tree ``_pgdist_C.so``.
* ``pgdist.engine``   — static-plan executor (explicit fwd/bwd, preallocated
  buffers, hipGraph capture), trainer with the reference's log format.
* ``pgdist.parallel`` — bootstrap (mpirun / SLURM / torchrun env), RCCL
  bucketed gradient all-reduce overlapped with backward, sharded sampler.
* ``pgdist.data``     — CIFAR-10 readers (native C++ binary reader), synthetic
  source, device-resident dataset.
* ``pgdist.serve``    — ``predict_cifar10_image`` and the web demo (port 7861).
"""

__version__ = "0.1.0"

CIFAR10_CLASSES = ('airplane', 'automobile', 'bird', 'cat', 'deer',
                   'dog', 'frog', 'horse', 'ship', 'truck')

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)
