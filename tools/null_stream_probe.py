"""Is work queued on the NULL stream ordered before a kernel on a non-blocking stream launched after it?

Round 2's renderer cleared its lazily allocated histogram scratch with hipMemset (null stream) from inside the
second lane's pass, then launched sky_compose (which bins into the scratch) on that non-blocking lane. This probe
reproduces the shape: the null stream is kept busy by a spin kernel (checked: the stream reports busy), then
  A: hipMemset(buf, 0)                 (the round-2 clear)
  B: a fill kernel on the null stream  (any stream-ordered clear on the null stream)
is queued behind it, and a copy of buf runs on a non-blocking stream. If the copy sees the old contents, the clear
was not ordered before it. Prints the host time of each enqueue and what the copy saw."""
import ctypes as C
import time

import torch


def case(name, clear, dev, hip):
    n = 1 << 16
    buf = torch.full((n,), 7, dtype=torch.int32, device=dev)
    out = torch.zeros_like(buf)
    torch.cuda.synchronize()
    side = torch.cuda.Stream(device=dev)                       # PyTorch streams are non-blocking
    null = torch.cuda.ExternalStream(0, device=dev)            # the legacy null stream
    with torch.cuda.stream(null):
        torch.cuda._sleep(400_000_000)                         # ~0.2 s of spinning on the null stream
    busy = not null.query()
    t0 = time.perf_counter()
    clear(buf, null, hip)
    t_clear = time.perf_counter() - t0
    with torch.cuda.stream(side):
        out.copy_(buf)
    side_done_early = False
    for _ in range(50):                                        # did the side copy finish while the null stream spun?
        if side.query():
            side_done_early = not null.query()
            break
        time.sleep(0.001)
    torch.cuda.synchronize()
    stale = int((out == 7).sum())
    print(f"{name}: null stream busy {busy}, enqueue host time {t_clear * 1e3:.2f} ms, side copy finished while the "
          f"null stream was still busy: {side_done_early}, copy saw {stale}/{n} stale words -> "
          f"{'NOT ordered after the null-stream clear' if stale else 'ordered'}", flush=True)


def memset_clear(buf, null, hip):
    assert hip.hipMemset(C.c_void_p(buf.data_ptr()), C.c_int(0), C.c_size_t(buf.numel() * 4)) == 0


def kernel_clear(buf, null, hip):
    with torch.cuda.stream(null):
        buf.zero_()


def main():
    hip = C.CDLL("libamdhip64.so")
    dev = torch.device("cuda", 0)
    case("A hipMemset on the null stream", memset_clear, dev, hip)
    case("B fill kernel on the null stream", kernel_clear, dev, hip)


if __name__ == "__main__":
    main()
