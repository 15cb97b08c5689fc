"""Reference-compatible log lines (the observable API).

Formats are byte-compatible with the reference prints so existing log parsers
keep working; extra information (global accuracy, img/s) goes on separate
lines prefixed with ``[pgdist]``.
"""
import sys
import time


def emit(line: str = "", rank: int = 0, file=None):
    if rank == 0:
        print(line, file=file or sys.stdout, flush=True)


def device_line(device) -> str:                                    # cifar10_serial_mobilenet_224.py:20
    return f"Device: {getattr(device, 'type', device)}"


def download_line() -> str:                                        # cifar10_mpi_mobilenet_224.py:94
    return "Downloading CIFAR-10 (if not present)..."


def samples_lines(n_train: int, n_test: int):                      # :65-66
    return [f"Train samples: {n_train}", f"Test samples: {n_test}"]


def params_line(n: int) -> str:                                   # :80
    return f"Total parameters: {n}"


def ddp_banner():                                                  # cifar10_mpi_mobilenet_224.py:53-56
    return ["=" * 70, "MPI + DDP MobileNetV2 CIFAR-10 (224x224)", "=" * 70]


def backend_line(backend: str, world: int, device) -> str:        # :61-62
    return f"Backend: {backend}, World size: {world}, Device(rank0): {device}"


def serial_epoch_line(e, E, t, train_loss, train_acc, test_loss, test_acc) -> str:   # serial :134-141
    return (f"Epoch {e}/{E} Time: {t:.2f}s Train Loss: {train_loss:.4f} Train Acc: {train_acc:.4f} "
            f"Test Loss: {test_loss:.4f} Test Acc: {test_acc:.4f}")


def ddp_epoch_line(e, E, t, train_loss, test_loss, test_acc_local) -> str:         # mpi :229-236
    return (f"Epoch {e}/{E} Time: {t:.2f}s Train Loss: {train_loss:.4f} Test Loss: {test_loss:.4f} "
            f"Test Acc(local): {test_acc_local:.4f}")


def best_line(acc: float, ddp: bool) -> str:
    return f"Best local test accuracy: {acc:.4f}" if ddp else f"Best test accuracy: {acc:.4f}"


def total_time_line(t: float) -> str:
    return f"Total training time: {t:.2f}s ({t / 60:.2f} min)"


def saved_line(path: str) -> str:
    return f"Saved {path}"


class Timer:
    def __init__(self):
        self.t0 = time.time()

    def elapsed(self) -> float:
        return time.time() - self.t0
