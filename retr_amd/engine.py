"""Train / eval entry points with the reference signatures (engine.py).

``pack_encoder_inputs`` (:20-48), ``train_one_epoch`` (:52-87), ``evaluate`` (:89-114) and
``eval_model`` (:125-187) keep their contracts so ``main.py`` / ``eval_model.py`` drop in.
Differences (all on the MI355X path, none observable in results):
  * ``nlgeval`` is imported lazily inside ``eval_model`` (the reference imports it at module
    top, ``engine.py:14-17``, which makes the module unimportable without the submodule);
  * under data parallelism (``retr_amd.ddp``) gradients are all-reduced before clipping, and
    the non-finite-loss exit is agreed over ranks (one all-reduce of a flag per step).
"""
import math
import sys
from collections import defaultdict
from os.path import abspath, dirname, join

import torch
import tqdm

from .models.utils import NestedTensor
from .eval_utils.decode import greedy_decoding


def pack_encoder_inputs(encoder_input, global_features, location_features, device="cpu"):
    if not global_features and not location_features:
        t_img, t_mask = encoder_input
        return (NestedTensor(t_img, t_mask).to(device),)
    if global_features and not location_features:
        t_img, t_mask, g_img, g_mask = encoder_input
        return (NestedTensor(t_img, t_mask).to(device), NestedTensor(g_img, g_mask).to(device))
    if not global_features and location_features:
        t_img, t_mask, l_feats = encoder_input
        return (NestedTensor(t_img, t_mask).to(device), l_feats.to(device))
    t_img, t_mask, g_img, g_mask, l_feats = encoder_input
    return (NestedTensor(t_img, t_mask).to(device), NestedTensor(g_img, g_mask).to(device),
            l_feats.to(device))


def clip_and_step(model, optimizer, max_norm):
    """engine.py:80-83: clip_grad_norm_(model.parameters(), max_norm) + optimizer.step().
    With a FusedAdamW that manages every trainable parameter both run as two fused kernels."""
    from .optim import FusedAdamW
    if isinstance(optimizer, FusedAdamW) and optimizer.covers(model.parameters()):
        optimizer.step(max_norm=max_norm if max_norm > 0 else 0.0)
        return
    if max_norm > 0:
        torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm)
    optimizer.step()


def forward_backward(model, criterion, samples, caps, cap_masks, optimizer):
    """engine.py:70-79: forward, CE loss, zero_grad, backward (no host sync)."""
    from . import ops
    ops.bump_seed()
    with ops.train_step_scope():
        outputs = model(*samples, caps[:, :-1], cap_masks[:, :-1])
        loss = criterion(outputs.permute(0, 2, 1), caps[:, 1:])
    optimizer.zero_grad()
    loss.backward()
    ops.flush_wgrad()            # no-op: backward's final callback already ran the queue
    return loss


def train_step(model, criterion, samples, caps, cap_masks, optimizer, max_norm, grad_sync=None):
    """One reference training step (engine.py:70-83) — returns the loss tensor (no host sync)."""
    loss = forward_backward(model, criterion, samples, caps, cap_masks, optimizer)
    if grad_sync is not None:
        grad_sync.synchronize()
    clip_and_step(model, optimizer, max_norm)
    return loss


class GraphedTrainStep:
    """The training step of ``train_step`` captured once into a hipGraph and replayed.

    Every kernel of the step (forward, CE, backward, gradient clipping and the optimizer) is
    stream-ordered and allocation-free inside the capture (torch's graph memory pool), so one
    ``hipGraphLaunch`` replaces ~1.2k individual launches and the Python/ctypes host work.
    Inputs are copied into static device buffers before each replay; dropout masks change
    every replay through the device-side step seed (ops.bump_seed inside the graph).

    First call: ``warmup`` eager steps (kernel attributes, weight copies, optimizer state
    allocation), then the parameters, optimizer state and step seed are restored to their
    values before the warm-up, the step is captured and replayed once -- so every call,
    the first included, applies exactly one update (one reference step) to its batch.
    After every replay the trainable parameters' autograd versions are bumped (the kernels
    write them through raw pointers) so version-keyed caches (bf16 weight copies, packed
    convolution weights, captured decode graphs) never serve values from before the replay,
    and FusedAdamW's host step counters advance with the device counter.

    Data parallel (``grad_sync``): forward + backward is captured as a chain of SEGMENT graphs
    cut where a gradient bucket becomes complete (the bucket's last post-accumulate-grad hook
    ends the running capture and begins the next, on the same capture stream and memory
    pool), then clip + optimizer as one more graph.  A replay runs segment 0, enqueues the RCCL
    all-reduce (AVG, in place on FusedAdamW's gradient arena) of every bucket that completed
    in it, runs segment 1 -- concurrently with those all-reduces on RCCL's stream -- and so on;
    the optimizer graph waits for every bucket.  No collective is captured inside a graph, so
    the all-reduces stay plain eager RCCL calls (the same ones the eager hook path issues)
    while still overlapping the rest of backward.  ``order`` records the replay's enqueue
    sequence (("segment", k) / ("allreduce", bucket)) for tests.

    Requirements: ``optimizer`` built with ``capturable=True`` (or a retr_amd FusedAdamW, whose
    step counter and lr live on the device); fixed batch shapes.
    """

    def __init__(self, model, criterion, optimizer, max_norm, grad_sync=None, warmup=2,
                 consume=True):
        self.model, self.criterion, self.optimizer = model, criterion, optimizer
        self.max_norm, self.grad_sync, self.warmup = max_norm, grad_sync, warmup
        # FusedAdamW consume mode inside the captured update (see __call__); False keeps the
        # step's gradients in the arena after each replay (tests read them), at the cost of
        # one zero fill of the arena before every replay
        self.consume = bool(consume)
        self.graph = None
        self.graph_opt = None
        self.segments = []        # DP: forward/backward segment graphs (segments[0] is graph)
        self.after = []           # DP: buckets whose all-reduce follows segment k
        self.order = []           # DP: enqueue order of the last replay
        self.schedule = None      # DP: the cross-rank-checked schedule (ddp.check_schedule)
        self.static = None
        self.loss = None
        self._active = None
        self._cap_stream = None
        self._tick = None

    def _step(self):
        s_img, s_mask, s_caps, s_cm = self.static
        return train_step(self.model, self.criterion, (NestedTensor(s_img, s_mask),), s_caps,
                          s_cm, self.optimizer, self.max_norm, self.grad_sync)

    def _fb(self):
        s_img, s_mask, s_caps, s_cm = self.static
        return forward_backward(self.model, self.criterion, (NestedTensor(s_img, s_mask),),
                                s_caps, s_cm, self.optimizer)

    def _capture(self):
        # thread-local capture: other threads' HIP calls stay legal meanwhile (the RCCL
        # process-group watchdog polls its work events from its own thread)
        mode = "thread_local"
        self.graph = torch.cuda.CUDAGraph()
        if self.grad_sync is None:
            with torch.cuda.graph(self.graph, capture_error_mode=mode):
                self.loss = self._step().detach()
            return
        self._capture_segmented()

    def _capture_segmented(self):
        """Forward + backward as segment graphs cut at bucket completions (see class doc).
        A cut happens inside a post-accumulate-grad hook, i.e. on autograd's device thread,
        while the main thread began the capture: "relaxed" capture mode is the one that lets a
        capture end on another thread than the one that began it."""
        import gc
        gs = self.grad_sync
        defer = gs.defer
        dev = torch.device("cuda", torch.cuda.current_device())
        self._tick = torch.zeros(1, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        gc.collect()
        torch.cuda.empty_cache()
        cs = self._cap_stream = torch.cuda.Stream(device=dev)
        cs.wait_stream(torch.cuda.current_stream())
        gs.defer = True                      # hooks only route gradients while capturing
        gs.on_ready = self._cut
        self.segments, self.after = [self.graph], [[]]
        self._pool = torch.cuda.graph_pool_handle()   # shared by every segment + the optimizer
        capturing = False
        try:
            with torch.cuda.stream(cs):
                self.graph.capture_begin(pool=self._pool, capture_error_mode="relaxed")
                capturing = True
                self.loss = self._fb().detach()
                capturing = False
                self.segments[-1].capture_end()
        except BaseException:
            if capturing:                    # leave no stream capturing behind the error
                with torch.cuda.stream(cs):
                    try:
                        self.segments[-1].capture_end()
                    except Exception:
                        pass
            gs.defer = defer
            raise
        finally:
            gs.on_ready = None
        torch.cuda.current_stream().wait_stream(cs)
        # every rank must have cut at the same buckets, or the replays would issue mismatched
        # collectives: all-gather the schedules and raise on a difference (ddp.check_schedule)
        self.schedule = gs.check_schedule(self.after)
        try:
            gs.synchronize()                 # eager: p.grad -> bucket views for the last graph
            self.graph_opt = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph_opt, pool=self._pool, stream=cs,
                                  capture_error_mode="thread_local"):
                clip_and_step(self.model, self.optimizer, self.max_norm)
        finally:
            gs.defer = defer

    def _cut(self, bucket):
        """Bucket ``bucket`` is complete: end the running segment (its all-reduce will follow
        that segment's replay) and begin the next one."""
        with torch.cuda.stream(self._cap_stream):
            self.segments[-1].capture_end()
            self.after[-1].append(bucket)
            g = torch.cuda.CUDAGraph()
            g.capture_begin(pool=self._pool, capture_error_mode="relaxed")
            self.segments.append(g)
            self.after.append([])
            self._tick.zero_()               # one node, so no segment is ever empty

    def _params(self):
        return [p for g in self.optimizer.param_groups for p in g["params"]]

    def _snapshot(self):
        from . import ops
        from .optim import FusedAdamW
        opt = self.optimizer
        seed = ops.seed_base().clone()
        if isinstance(opt, FusedAdamW):
            return ("fused", opt.snapshot(), seed)
        params = [p.detach().clone() for p in self._params()]
        state = {id(p): {k: (v.clone() if torch.is_tensor(v) else v)
                         for k, v in opt.state[p].items()} for p in self._params()
                 if p in opt.state}
        return ("torch", (params, state), seed)

    @torch.no_grad()
    def _restore(self, snap):
        from . import ops
        kind, data, seed = snap
        opt = self.optimizer
        ops.seed_base().copy_(seed)
        if kind == "fused":
            opt.restore(data)
        else:
            params, state = data
            for p, v in zip(self._params(), params):
                p.copy_(v)
            for p in self._params():
                st = opt.state.get(p)
                if not st:
                    continue
                old = state.get(id(p))
                for k, v in st.items():
                    if not torch.is_tensor(v):
                        continue
                    if old is None:           # state created by the warm-up: back to "fresh"
                        v.zero_()
                    else:
                        v.copy_(old[k])
        self._bump()

    def _clean_arena(self):
        """The captured step expects a zero gradient arena (its own update leaves it so): an
        eager step run since the last replay without consume mode left gradients in it."""
        a = getattr(self.optimizer, "arena", None)
        if a is not None and a.dirty:
            a.G.zero_()
            a.dirty = False

    def _bump(self):
        inc = torch.autograd.graph.increment_version
        for p in self._params():
            if p.requires_grad:
                inc(p)
        if hasattr(self.optimizer, "mark_shadow_fresh") and self._active:
            # the captured update rewrote the bf16 shadow of every parameter it stepped
            self.optimizer.mark_shadow_fresh(self._active)

    def input_buffers(self):
        """The captured step's static inputs (images, image mask, captions, caption mask), set
        by the first call: a loader that writes each batch into them and passes them back
        saves the per-step device-to-device staging copy (78.6 MB of images at cfg2)."""
        return self.static

    def __call__(self, samples, caps, cap_masks):
        nt = samples[0]
        if self.static is None:
            self.static = (nt.tensors.clone(), nt.mask.clone(), caps.clone(), cap_masks.clone())
        else:
            for dst, src in zip(self.static, (nt.tensors, nt.mask, caps, cap_masks)):
                # zero-copy when the caller handed back the step's own input buffers (a loader
                # that writes each batch into input_buffers()): nothing to stage
                if (src.data_ptr() != dst.data_ptr() or src.shape != dst.shape
                        or src.stride() != dst.stride() or src.dtype != dst.dtype):
                    dst.copy_(src, non_blocking=True)
        if self.graph is None:
            opt = self.optimizer
            consume0 = getattr(opt, "consume_grads", None)
            if consume0 is not None:
                # FusedAdamW consume mode (its update zeroes the gradient arena: no zero fill
                # per replay) only for the steps this object runs -- warm-up and capture; the
                # captured update keeps it on every replay, eager steps outside keep the
                # optimizer's own setting (p.grad holds the clipped gradient after step())
                opt.consume_grads = self.consume
            try:
                snap = self._snapshot()
                side = torch.cuda.Stream()
                side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(side):
                    for _ in range(self.warmup):
                        self._step().detach()
                torch.cuda.current_stream().wait_stream(side)
                torch.cuda.synchronize()
                opt.zero_grad(set_to_none=True)
                self._capture()
                self._active = list(getattr(opt, "_last_active", []))
                self._restore(snap)
            finally:
                if consume0 is not None:
                    opt.consume_grads = consume0
        else:
            self._clean_arena()
        if hasattr(self.optimizer, "sync_hyper"):
            self.optimizer.sync_hyper()      # lr schedule changes reach the captured kernels
        if self.graph_opt is None:
            self.graph.replay()
        else:
            gs = self.grad_sync
            self.order = []
            for k, g in enumerate(self.segments):
                g.replay()
                self.order.append(("segment", k))
                for b in self.after[k]:
                    gs._launch(b)            # RCCL stream waits for segment k only
                    self.order.append(("allreduce", b))
            gs.synchronize()                 # any bucket not launched yet; stream waits on all
            self.graph_opt.replay()
        if hasattr(self.optimizer, "_advance_host"):
            self.optimizer._advance_host(self._active)
        self._bump()
        return self.loss


def train_one_epoch(model, criterion, data_loader, optimizer, device, epoch, max_norm,
                    grad_sync=None):
    from . import ops
    model.train()
    criterion.train()
    epoch_loss = 0.0
    total = len(data_loader)
    global_features = data_loader.dataset.return_global_context
    location_features = data_loader.dataset.return_location_features
    with tqdm.tqdm(total=total) as pbar:
        for ann_ids, *encoder_input, caps, cap_masks in data_loader:
            samples = pack_encoder_inputs(encoder_input, global_features, location_features,
                                          device)
            caps = caps.to(device)
            cap_masks = cap_masks.to(device)
            with ops.train_step_scope():
                outputs = model(*samples, caps[:, :-1], cap_masks[:, :-1])
                loss = criterion(outputs.permute(0, 2, 1), caps[:, 1:])
            loss_value = loss.item()
            epoch_loss += loss_value
            finite = math.isfinite(loss_value)
            if grad_sync is not None:
                # every rank takes the same decision: a rank that exits alone would leave the
                # others blocked in the gradient all-reduce of this step
                finite = grad_sync.all_finite(finite)
            if not finite:
                print(f"Loss is {loss_value}, stopping training")
                sys.exit(1)
            optimizer.zero_grad()
            loss.backward()
            if grad_sync is not None:
                grad_sync.synchronize()
            clip_and_step(model, optimizer, max_norm)
            pbar.update(1)
    return epoch_loss / total


@torch.no_grad()
def evaluate(model, criterion, data_loader, device):
    model.eval()
    criterion.eval()
    validation_loss = 0.0
    total = len(data_loader)
    global_features = data_loader.dataset.return_global_context
    location_features = data_loader.dataset.return_location_features
    with tqdm.tqdm(total=total) as pbar:
        for ann_ids, *encoder_input, caps, cap_masks in data_loader:
            samples = pack_encoder_inputs(encoder_input, global_features, location_features,
                                          device)
            caps = caps.to(device)
            cap_masks = cap_masks.to(device)
            outputs = model(*samples, caps[:, :-1], cap_masks[:, :-1])
            loss = criterion(outputs.permute(0, 2, 1), caps[:, 1:])
            validation_loss += loss.item()
            pbar.update(1)
    return validation_loss / total


def normalize_with_tokenizer(sent, tokenizer):
    return tokenizer.decode(tokenizer.encode(sent), skip_special_tokens=True)


def _nlgeval():
    """Lazy import of the nlgeval submodule (reference engine.py:14-17)."""
    try:
        from nlgeval import NLGEval  # noqa
    except ImportError:
        sys.path.append(join(dirname(abspath(__file__)), "nlgeval"))
        from nlgeval import NLGEval  # noqa
    return NLGEval


def eval_model(model, data_loader, tokenizer, config, metrics_to_omit=[], print_samples=False):
    """Decode the loader with greedy decoding and score with nlgeval (engine.py:125-187)."""
    model.eval()
    NLGEval = _nlgeval()
    nlgeval = NLGEval(no_skipthoughts=True, no_glove=True, metrics_to_omit=metrics_to_omit)
    annotations = defaultdict(list)
    for a in data_loader.dataset.annot:
        annotations[a[0]].append(a[2])
    hypotheses, ids_hypotheses, references = [], [], []
    pad_id = tokenizer.convert_tokens_to_ids(tokenizer.pad_token)
    bos_id = tokenizer.convert_tokens_to_ids(tokenizer.cls_token)
    eos_id = tokenizer.convert_tokens_to_ids(tokenizer.sep_token)
    global_features = data_loader.dataset.return_global_context
    location_features = data_loader.dataset.return_location_features
    for i, (ann_ids, *encoder_input, caps, cap_masks) in enumerate(tqdm.tqdm(data_loader)):
        samples = pack_encoder_inputs(encoder_input, global_features, location_features)
        hyps = greedy_decoding(samples, model, tokenizer, max_len=config.max_position_embeddings,
                               clean=True, pad_token=pad_id, bos_token=bos_id,
                               eos_token=eos_id, device="auto")
        hypotheses += hyps
        ids_hyps = [{"ann_id": i, "expression": h} for i, h in zip(ann_ids.tolist(), hyps)]
        ids_hypotheses += ids_hyps
        if print_samples:
            print(*ids_hyps, sep="\n")
        refs = [annotations[i.item()] for i in ann_ids]
        references += [[normalize_with_tokenizer(r, tokenizer) for r in _refs] for _refs in refs]
    transposed_references = list(map(list, zip(*references)))
    metrics_dict = nlgeval.compute_metrics(ref_list=transposed_references, hyp_list=hypotheses)
    return metrics_dict, ids_hypotheses
