"""Multi-GPU sharding of a codec batch.

Every batch element is compressed independently with its own statistics
and archive (reference README.md:110; ans/GpuANSEncode.cuh:686-711), so a
batch shards by contiguous element ranges with no data-path collective:
one process per GPU runs the full codec on its local HBM.  The only
exchange is an all-gather of the per-element compressed sizes -- RCCL over
xGMI on MI355X (backend "nccl"), gloo in the CPU tests -- from which every
rank derives the global packing offsets of the archives.
"""
import torch
import torch.distributed as dist


def shard_range(nb, rank, world):
    """Contiguous [start, stop) of ceil(nb / world) elements for `rank`."""
    per = -(-nb // world)
    start = min(nb, rank * per)
    return start, min(nb, start + per)


def gather_sizes(local_sizes, nb, group=None):
    """All-gather per-element compressed sizes (int32, one per local element)
    into the global [nb] vector (int64).  Shards are padded to the common
    per-rank length so a single all_gather_into_tensor suffices."""
    world = dist.get_world_size(group)
    per = -(-nb // world)
    buf = torch.zeros(per, dtype=torch.int32, device=local_sizes.device)
    buf[: local_sizes.numel()] = local_sizes.to(torch.int32)
    out = torch.empty(per * world, dtype=torch.int32, device=local_sizes.device)
    dist.all_gather_into_tensor(out, buf, group=group)
    return out[:nb].to(torch.int64)


def archive_offsets(sizes, align=16):
    """Exclusive prefix of roundUp(size, align): where each element's archive
    lands when the batch is packed back to back (archives are 16 B aligned,
    SURVEY 8(b))."""
    r = (sizes + (align - 1)) // align * align
    return torch.cumsum(r, 0) - r


class GpuFloatCodec:
    """The float codec on the local GPU (ops.compress_data /
    ops.decompress_data: k_pcompress or k_hist -> k_encode, then k_decode) for the compressed collectives."""

    def __init__(self, checksum=False):
        self.checksum = checksum

    def compress(self, tensors):
        from . import ops

        comp, sizes, _ = ops.compress_data(True, tensors, self.checksum)
        return comp, sizes

    def decompress(self, archives, outs):
        from . import ops

        status = torch.empty(len(archives), dtype=torch.uint8, device=outs[0].device)
        ops.decompress_data(True, archives, outs, self.checksum, out_status=status)
        if not bool((status != 0).all()):
            raise RuntimeError("compressed collective: an archive failed to decode")


def _check_sizes(sizes, what):
    """Archive sizes seen by every rank: 0 marks an element whose compression
    was abandoned (a bounded cross-workgroup wait ran out, see
    dietgpu_device_error_count); no valid archive is shorter than its headers.
    Raising here, where every rank sees the same sizes, keeps the ranks in
    step (a zero-length slot would otherwise alias the next archive and could
    decode into the wrong output)."""
    bad = (torch.as_tensor(sizes) <= 0).nonzero().view(-1).tolist()
    if bad:
        raise RuntimeError(f"{what}: compression of element(s) {bad[:8]} was abandoned (archive size 0)")


def _pack(comp, sizes, offs, length, dev):
    """Pack the archive rows comp[i, :sizes[i]] back to back at the 16 B
    aligned offsets `offs` (= archive_offsets(sizes)) into a buffer of
    `length` bytes: one masked gather over the [nb, cols] archive matrix (the
    16 B tails of each row ride along as don't-care padding), no per-element
    launches."""
    nb, cols = comp.shape
    if cols % 16:
        comp = torch.nn.functional.pad(comp, (0, 16 - cols % 16))
        cols = comp.shape[1]
    padded = ((sizes.to(torch.int64) + 15) // 16 * 16).to(comp.device)
    if nb:
        expect = torch.cumsum(padded.cpu(), 0) - padded.cpu()
        assert torch.equal(expect, torch.as_tensor(offs, dtype=torch.int64).cpu()), \
            "_pack: offsets must be the 16 B aligned exclusive prefix of the sizes"
    buf = torch.zeros(max(int(length), 16), dtype=torch.uint8, device=dev)
    mask = torch.arange(cols, device=comp.device)[None, :] < padded[:, None]
    flat = comp[mask]
    buf[: flat.numel()] = flat.to(dev)
    return buf


def all_gather_compressed(tensors, group=None, codec=None):
    """All-gather a list of float tensors in compressed form (SURVEY.md 8(f)
    rank 3: the compressed collectives the reference was built for,
    README.md:94-96).

    Every rank passes the same number k of tensors of one float dtype (shapes
    may differ between ranks).  Each rank compresses its tensors locally, the
    ranks all-gather (numel, archive size) per tensor, then ONE
    all_gather_into_tensor moves the packed archives (each rank's slot is the
    largest per-rank packed size) and every rank decompresses all of them.
    Returns the flat decoded tensors rank-major: [rank 0's k, rank 1's, ...].
    The codec is lossless: the result equals an uncompressed all-gather bit
    for bit.
    """
    codec = codec or GpuFloatCodec()
    world = dist.get_world_size(group)
    k = len(tensors)
    if k == 0:
        return []
    dtype, dev = tensors[0].dtype, tensors[0].device
    flat = [t.contiguous().view(-1) for t in tensors]
    comp, sizes = codec.compress(flat)
    meta = torch.stack([torch.tensor([t.numel() for t in flat], dtype=torch.int64),
                        sizes.to("cpu", torch.int64)]).to(dev)
    allmeta = torch.empty(world * 2 * k, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(allmeta, meta.view(-1), group=group)
    allmeta = allmeta.view(world, 2, k).cpu()
    asizes = allmeta[:, 1, :]
    _check_sizes(asizes.reshape(-1), "all_gather_compressed")
    offs = archive_offsets(asizes.reshape(-1)).view(world, k)
    offs = offs - offs[:, :1]  # per-rank packing, from 0
    packed = offs[:, -1] + (asizes[:, -1] + 15) // 16 * 16
    span = max(int(packed.max()), 16)
    rank = dist.get_rank(group)
    send = _pack(comp, asizes[rank], offs[rank], span, dev)
    recv = torch.empty(world * span, dtype=torch.uint8, device=dev)
    dist.all_gather_into_tensor(recv, send, group=group)
    archives, outs = [], []
    for r in range(world):
        for i in range(k):
            o = r * span + int(offs[r, i])
            archives.append(recv[o:o + int(asizes[r, i])])
            outs.append(torch.empty(int(allmeta[r, 0, i]), dtype=dtype, device=dev))
    codec.decompress(archives, outs)
    return outs


def all_to_all_compressed(tensors, group=None, codec=None):
    """All-to-all of float tensors in compressed form: tensors[j] (one float
    dtype, any sizes) goes to rank j; returns the world tensors received,
    tensor r from rank r (flat).  This rank's outgoing tensors are compressed
    in one batch, the (numel, size) pairs are exchanged with one small
    all_to_all_single, the packed archives with one all_to_all_single whose
    split sizes are the packed lengths."""
    codec = codec or GpuFloatCodec()
    world = dist.get_world_size(group)
    if len(tensors) != world:
        raise ValueError("all_to_all_compressed: one tensor per destination rank")
    dtype, dev = tensors[0].dtype, tensors[0].device
    flat = [t.contiguous().view(-1) for t in tensors]
    comp, sizes = codec.compress(flat)
    sizes = sizes.to("cpu", torch.int64)
    lens = (sizes + 15) // 16 * 16
    send = _pack(comp, sizes, torch.cumsum(lens, 0) - lens, int(lens.sum()), dev)
    meta = torch.stack([torch.tensor([t.numel() for t in flat], dtype=torch.int64), sizes],
                       dim=1).to(dev)  # row j goes to rank j
    # every rank gathers the whole (source, destination) table, so a poisoned
    # archive anywhere raises on every rank before the payload exchange
    allmeta = torch.empty([world * world, 2], dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(allmeta, meta, group=group)
    allmeta = allmeta.view(world, world, 2).cpu()
    _check_sizes(allmeta[:, :, 1].reshape(-1), "all_to_all_compressed")
    rmeta = allmeta[:, dist.get_rank(group), :]
    rlens = (rmeta[:, 1] + 15) // 16 * 16
    recv = torch.empty(max(int(rlens.sum()), 16), dtype=torch.uint8, device=dev)
    dist.all_to_all_single(recv[: int(rlens.sum())], send[: int(lens.sum())],
                           output_split_sizes=rlens.tolist(), input_split_sizes=lens.tolist(),
                           group=group)
    roffs = torch.cumsum(rlens, 0) - rlens
    archives = [recv[int(roffs[r]):int(roffs[r]) + int(rmeta[r, 1])] for r in range(world)]
    outs = [torch.empty(int(rmeta[r, 0]), dtype=dtype, device=dev) for r in range(world)]
    codec.decompress(archives, outs)
    return outs
