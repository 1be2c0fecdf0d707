// Package gpusched is the Go side of the MI355X scheduling core: it packs the informer snapshot of
// v1.Node and v1.Pod objects into the SoA columns libminisched_hip.so reads and calls its C-ABI
// (include/minisched_hip.h) through cgo.
//
// It replaces the selection part of Scheduler.scheduleOne (minisched/minisched.go:40-87: the node
// LIST, RunFilterPlugins, RunPreScorePlugins, RunScorePlugins and selectHost) for a batch of pods
// drained from activeQ. Permit, Bind, the queue and the event handlers stay in Go, unchanged.
//
// The framework.*Plugin values stay the source of truth: New maps their Name()s to device plugin
// ids and reports ErrUnsupported for a plugin list the device path does not implement, in which
// case the caller keeps the reference's per-pod Go loop (minisched.go:115-199).
//
// Not compiled in the repository that ships this file (its build image has no Go toolchain): copy
// the go/minisched tree into the reference's minisched/ and build it with the module's own go.mod
// (k8s.io/kubernetes v1.22.0). See go/README.md.
package gpusched

/*
#cgo CFLAGS: -I${SRCDIR}/../../../include
#cgo LDFLAGS: -L${SRCDIR}/../../../mini-kube-scheduler_amd -lminisched_hip -Wl,-rpath,${SRCDIR}/../../../mini-kube-scheduler_amd
#include <stdlib.h>
#include "minisched_hip.h"
*/
import "C"

import (
	"errors"
	"fmt"
	"runtime"
	"sort"
	"sync"
	"unsafe"

	v1 "k8s.io/api/core/v1"
	"k8s.io/apimachinery/pkg/labels"
	"k8s.io/apimachinery/pkg/util/sets"
	corelisters "k8s.io/client-go/listers/core/v1"
	"k8s.io/client-go/tools/cache"
	"k8s.io/kubernetes/pkg/scheduler/framework"
)

// ErrUnsupported: the plugin list names a plugin with no device implementation. The caller keeps
// the reference's Go loop for it.
var ErrUnsupported = errors.New("gpusched: plugin list not implemented on the device")

// Device ids of the framework.Plugin names the device path implements (initialize.go:80-123).
var (
	filterIDs   = map[string]C.int32_t{"NodeUnschedulable": C.MSH_PLUGIN_NODE_UNSCHEDULABLE}
	preScoreIDs = map[string]C.int32_t{"NodeNumber": C.MSH_PLUGIN_NODE_NUMBER}
	scoreIDs    = map[string]C.int32_t{"NodeNumber": C.MSH_PLUGIN_NODE_NUMBER}
)

// Normalize is the NormalizeScore stage of one score plugin (msh_normalize). NodeNumber has no
// ScoreExtensions (nodenumber.go:98-100): NormalizeNone reproduces the reference.
type Normalize int32

const (
	NormalizeNone           Normalize = C.MSH_NORMALIZE_NONE
	NormalizeDefault        Normalize = C.MSH_NORMALIZE_DEFAULT         // helper.DefaultNormalizeScore(100, false)
	NormalizeDefaultReverse Normalize = C.MSH_NORMALIZE_DEFAULT_REVERSE // helper.DefaultNormalizeScore(100, true)
	NormalizeMinMax         Normalize = C.MSH_NORMALIZE_MINMAX
)

// ScoreConfig is one entry of the score list. The reference has no weights ("TODO: plugin weight",
// minisched.go:187): Weight 1 reproduces it.
type ScoreConfig struct {
	Plugin    framework.ScorePlugin
	Weight    int64
	Normalize Normalize
}

// Scores is the reference's score list as device entries: weight 1, no normalize (minisched.go:164-199).
func Scores(plugins []framework.ScorePlugin) []ScoreConfig {
	out := make([]ScoreConfig, len(plugins))
	for i, p := range plugins {
		out[i] = ScoreConfig{Plugin: p, Weight: 1, Normalize: NormalizeNone}
	}
	return out
}

// Ctx is one device context (one per GPU; not safe for concurrent use: give each goroutine that
// submits its own Ctx, locked to its OS thread or not — every entry point sets the device).
type Ctx struct {
	c        *C.msh_ctx
	byIndex  []*v1.Node // device node index -> node (List order)
	hasNodes bool
}

func (x *Ctx) lastErr(what string, rc C.int) error {
	return fmt.Errorf("%s: %d: %s", what, int(rc), C.GoString(C.msh_last_error(x.c)))
}

// New creates a device context for `device` and installs the plugin lists (Scheduler.filterPlugins,
// preScorePlugins, scorePlugins; initialize.go:25-27).
func New(device int, filters []framework.FilterPlugin, preScores []framework.PreScorePlugin, scores []ScoreConfig) (*Ctx, error) {
	fids := make([]C.int32_t, 0, len(filters))
	for _, p := range filters {
		id, ok := filterIDs[p.Name()]
		if !ok {
			return nil, fmt.Errorf("%w: filter %q", ErrUnsupported, p.Name())
		}
		fids = append(fids, id)
	}
	pids := make([]C.int32_t, 0, len(preScores))
	for _, p := range preScores {
		id, ok := preScoreIDs[p.Name()]
		if !ok {
			return nil, fmt.Errorf("%w: pre-score %q", ErrUnsupported, p.Name())
		}
		pids = append(pids, id)
	}
	sids := make([]C.int32_t, 0, len(scores))
	ws := make([]C.int64_t, 0, len(scores))
	norms := make([]C.int32_t, 0, len(scores))
	for _, s := range scores {
		id, ok := scoreIDs[s.Plugin.Name()]
		if !ok {
			return nil, fmt.Errorf("%w: score %q", ErrUnsupported, s.Plugin.Name())
		}
		w := s.Weight
		if w == 0 {
			w = 1
		}
		sids = append(sids, id)
		ws = append(ws, C.int64_t(w))
		norms = append(norms, C.int32_t(s.Normalize))
	}
	var c *C.msh_ctx
	if rc := C.msh_create(C.int(device), &c); rc != C.MSH_OK {
		return nil, fmt.Errorf("msh_create(%d): %d: %s", device, int(rc), C.GoString(C.msh_last_error(nil)))
	}
	x := &Ctx{c: c}
	if rc := C.msh_set_plugins_ex(c, ptrI32(fids), C.int32_t(len(fids)), ptrI32(pids), C.int32_t(len(pids)),
		ptrI32(sids), ptrI64(ws), ptrI32(norms), C.int32_t(len(sids))); rc != C.MSH_OK {
		err := x.lastErr("msh_set_plugins_ex", rc)
		C.msh_destroy(c)
		return nil, err
	}
	runtime.SetFinalizer(x, (*Ctx).Close)
	return x, nil
}

// Close releases the device context. Batches in flight are waited for.
func (x *Ctx) Close() {
	if x.c != nil {
		C.msh_destroy(x.c)
		x.c = nil
	}
	runtime.SetFinalizer(x, nil)
}

// UploadNodes replaces the per-cycle Nodes().List (minisched.go:40): the nodes are put in List
// order (byte-sorted names, the apiserver's etcd key order) and their two columns uploaded.
// It returns the device-index -> node mapping, also kept for ScheduleBatch.
func (x *Ctx) UploadNodes(nodes []v1.Node) ([]*v1.Node, error) {
	sorted := make([]*v1.Node, len(nodes))
	for i := range nodes {
		sorted[i] = &nodes[i]
	}
	sort.Slice(sorted, func(a, b int) bool { return sorted[a].Name < sorted[b].Name }) // Go string order == bytes
	uns := make([]C.uint8_t, len(sorted))
	dig := make([]C.int8_t, len(sorted))
	for i, n := range sorted {
		if n.Spec.Unschedulable {
			uns[i] = 1
		}
		dig[i] = C.int8_t(suffixDigit(n.Name))
	}
	if rc := C.msh_upload_nodes(x.c, C.int32_t(len(sorted)), ptrU8(uns), ptrI8(dig)); rc != C.MSH_OK {
		return nil, x.lastErr("msh_upload_nodes", rc)
	}
	x.byIndex, x.hasNodes = sorted, true
	return sorted, nil
}

// UpdateNode applies an informer Update that keeps the node's name (eventhandler.go:45-50, e.g. a
// cordon flipping Spec.Unschedulable) in O(1) host->device traffic. Adds, deletes and renames
// change List positions: call UploadNodes for those.
func (x *Ctx) UpdateNode(n *v1.Node) error { return x.UpdateNodes([]*v1.Node{n}) }

// UpdateNodes is UpdateNode for several nodes in one msh_patch_nodes call.
func (x *Ctx) UpdateNodes(nodes []*v1.Node) error {
	if len(nodes) == 0 {
		return nil
	}
	idx := make([]C.int32_t, len(nodes))
	uns := make([]C.uint8_t, len(nodes))
	dig := make([]C.int8_t, len(nodes))
	for k, n := range nodes {
		i := sort.Search(len(x.byIndex), func(q int) bool { return x.byIndex[q].Name >= n.Name })
		if i == len(x.byIndex) || x.byIndex[i].Name != n.Name {
			return fmt.Errorf("gpusched: node %q is not in the uploaded snapshot", n.Name)
		}
		idx[k] = C.int32_t(i)
		if n.Spec.Unschedulable {
			uns[k] = 1
		}
		dig[k] = C.int8_t(suffixDigit(n.Name))
	}
	if rc := C.msh_patch_nodes(x.c, C.int32_t(len(nodes)), ptrI32(idx), ptrU8(uns), ptrI8(dig)); rc != C.MSH_OK {
		return x.lastErr("msh_patch_nodes", rc)
	}
	// Copy on write: a HostBatch in flight keeps the mapping (and the node objects) of the table version
	// it was launched on; the names and List positions are the same, so either decodes the same index.
	byIndex := append([]*v1.Node(nil), x.byIndex...)
	for k, n := range nodes {
		byIndex[idx[k]] = n
	}
	x.byIndex = byIndex
	return nil
}

// NodeSnapshot keeps a Ctx's node table in step with the Node informer (eventhandler.go:45-65)
// instead of a LIST per cycle (minisched.go:40): an Add or a Delete changes List positions and marks
// the table for one full upload; an Update of an existing name (a cordon flip, or any other field
// change) queues an O(1) patch. Sync brings the Ctx up to date before a batch. The handlers run on
// the informer's goroutine, Sync on the scheduling loop's: both take the lock. Register it next to
// the reference's own handlers (which requeue pods on Node events):
//
//	snap := gpusched.NewNodeSnapshot()
//	informerFactory.Core().V1().Nodes().Informer().AddEventHandler(snap.Handlers())
//
// The Python mirror is mini-kube-scheduler_amd/nodecache.py (NodeCache.sync).
//
// A structural upload reads the informer's store through its lister when one is given
// (NewNodeSnapshotFromLister): WaitForCacheSync (scheduler.go:72-75) returns once the store holds the
// initial LIST, which can be before the handlers have been called for all of it, so a map filled by
// the handlers alone could upload a partial node list for the first batches, where the reference's
// per-cycle LIST (minisched.go:40) always sees every node. Handler calls that arrive after such an
// upload for nodes it already holds are then Updates: patches of identical values.
type NodeSnapshot struct {
	mu         sync.Mutex
	lister     corelisters.NodeLister // the informer's store (nil: the handlers' map alone)
	nodes      map[string]*v1.Node
	structural bool                // List positions changed since the last Sync
	patched    map[string]*v1.Node // names updated in place since the last Sync
}

// NewNodeSnapshot starts empty and structurally dirty: the first Sync uploads.
func NewNodeSnapshot() *NodeSnapshot {
	return &NodeSnapshot{nodes: map[string]*v1.Node{}, structural: true, patched: map[string]*v1.Node{}}
}

// NewNodeSnapshotFromLister is NewNodeSnapshot whose structural uploads read the informer's store:
//
//	nodes := informerFactory.Core().V1().Nodes()
//	snap := gpusched.NewNodeSnapshotFromLister(nodes.Lister())
//	nodes.Informer().AddEventHandler(snap.Handlers())
func NewNodeSnapshotFromLister(l corelisters.NodeLister) *NodeSnapshot {
	s := NewNodeSnapshot()
	s.lister = l
	return s
}

// Handlers are the informer callbacks (a cache.ResourceEventHandler).
func (s *NodeSnapshot) Handlers() cache.ResourceEventHandlerFuncs {
	return cache.ResourceEventHandlerFuncs{AddFunc: s.OnAdd, UpdateFunc: s.OnUpdate, DeleteFunc: s.OnDelete}
}

// OnAdd: a new name is a structural change; an Add for a name already present is an Update.
func (s *NodeSnapshot) OnAdd(obj interface{}) {
	n, ok := obj.(*v1.Node)
	if !ok {
		return
	}
	s.mu.Lock()
	defer s.mu.Unlock()
	if _, had := s.nodes[n.Name]; had {
		s.nodes[n.Name] = n
		s.patched[n.Name] = n
		return
	}
	s.nodes[n.Name] = n
	s.structural = true
}

// OnUpdate: names are immutable, so an Update keeps the node's List position: a patch.
func (s *NodeSnapshot) OnUpdate(_, newObj interface{}) {
	n, ok := newObj.(*v1.Node)
	if !ok {
		return
	}
	s.mu.Lock()
	defer s.mu.Unlock()
	if _, had := s.nodes[n.Name]; !had {
		s.nodes[n.Name] = n
		s.structural = true
		return
	}
	s.nodes[n.Name] = n
	s.patched[n.Name] = n
}

// OnDelete: every later List position shifts: a structural change.
func (s *NodeSnapshot) OnDelete(obj interface{}) {
	var name string
	switch t := obj.(type) {
	case *v1.Node:
		name = t.Name
	case cache.DeletedFinalStateUnknown:
		n, ok := t.Obj.(*v1.Node)
		if !ok {
			return
		}
		name = n.Name
	default:
		return
	}
	s.mu.Lock()
	defer s.mu.Unlock()
	if _, had := s.nodes[name]; had {
		delete(s.nodes, name)
		delete(s.patched, name)
		s.structural = true
	}
}

// Sync brings x's device table up to date: "upload" (msh_upload_nodes of every node, after an Add
// or a Delete), "patch" (msh_patch_nodes of the updated nodes only) or "clean".
func (s *NodeSnapshot) Sync(x *Ctx) (string, error) {
	s.mu.Lock()
	defer s.mu.Unlock()
	if s.structural {
		if s.lister != nil { // the store, consistent with HasSynced, replaces what the handlers have seen
			listed, err := s.lister.List(labels.Everything())
			if err != nil {
				return "", err
			}
			s.nodes = make(map[string]*v1.Node, len(listed))
			for _, n := range listed {
				s.nodes[n.Name] = n
			}
		}
		all := make([]v1.Node, 0, len(s.nodes))
		for _, n := range s.nodes {
			all = append(all, *n)
		}
		if _, err := x.UploadNodes(all); err != nil {
			return "", err
		}
		s.structural = false
		s.patched = map[string]*v1.Node{}
		return "upload", nil
	}
	if len(s.patched) > 0 {
		upd := make([]*v1.Node, 0, len(s.patched))
		for _, n := range s.patched {
			upd = append(upd, n)
		}
		if err := x.UpdateNodes(upd); err != nil {
			return "", err
		}
		s.patched = map[string]*v1.Node{}
		return "patch", nil
	}
	return "clean", nil
}

// Result of scheduleOne's selection part (minisched.go:50-87) for one pod.
type Result struct {
	Node   *v1.Node            // set when placed (selectHost's choice: the first maximum in List order)
	Score  int64               // the selected node's total score
	FitErr *framework.FitError // RunFilterPlugins found no feasible node (minisched.go:143-148)
	Err    error               // a Score plugin failed (minisched.go:70-75); ErrorFunc gets the nil filter error
}

// HostBatch holds one batch's pod columns and outputs in page-locked C memory (msh_host_alloc), so
// msh_schedule_batch copies nothing on the host: the kernel reads the columns and writes the outputs
// over PCIe. It is C memory, so the cgo pointer rules do not apply to it. Allocate once, reuse.
type HostBatch struct {
	cap         int
	mem         unsafe.Pointer
	pd          []C.int8_t
	pt          []C.uint8_t
	idx, status []C.int32_t
	score       []C.int64_t
	ticket      C.uint64_t // the pending msh_schedule_batch_async ticket, 0 = none
	pods        []*v1.Pod
	byIndex     []*v1.Node // the Ctx's device index -> node mapping when the batch was launched
}

// NewHostBatch allocates a HostBatch for up to `cap` pods (18 B per pod).
func NewHostBatch(cap int) (*HostBatch, error) {
	var mem unsafe.Pointer
	// score | idx | status | digit | tol: 8-byte aligned sections
	if rc := C.msh_host_alloc(C.size_t(18*cap+16), &mem); rc != C.MSH_OK {
		return nil, fmt.Errorf("msh_host_alloc(%d pods): %d", cap, int(rc))
	}
	b := &HostBatch{cap: cap, mem: mem}
	base := uintptr(mem)
	b.score = unsafe.Slice((*C.int64_t)(unsafe.Pointer(base)), cap)
	b.idx = unsafe.Slice((*C.int32_t)(unsafe.Pointer(base+uintptr(8*cap))), cap)
	b.status = unsafe.Slice((*C.int32_t)(unsafe.Pointer(base+uintptr(12*cap))), cap)
	b.pd = unsafe.Slice((*C.int8_t)(unsafe.Pointer(base+uintptr(16*cap))), cap)
	b.pt = unsafe.Slice((*C.uint8_t)(unsafe.Pointer(base+uintptr(17*cap))), cap)
	runtime.SetFinalizer(b, func(b *HostBatch) { C.msh_host_free(b.mem) })
	return b, nil
}

// pack writes the pods' PreScore / Filter inputs: the name suffix digit (NodeNumber.PreScore,
// nodenumber.go:50-64) and whether the tolerations tolerate the unschedulable taint
// (NodeUnschedulable.Filter, upstream v1.22.0), and keeps the Ctx's current index -> node mapping:
// the launch reads the table version published now, so its indices decode against this mapping even
// if UploadNodes replaces it before Wait (an upload builds a new slice; UpdateNodes keeps names and
// positions).
func (x *Ctx) pack(b *HostBatch, pods []*v1.Pod) error {
	if len(pods) > b.cap {
		return fmt.Errorf("gpusched: batch of %d pods exceeds the HostBatch capacity %d", len(pods), b.cap)
	}
	for j, pod := range pods {
		b.pd[j] = C.int8_t(suffixDigit(pod.Name))
		b.pt[j] = 0
		if tolerates(pod.Spec.Tolerations) {
			b.pt[j] = 1
		}
	}
	b.pods = pods
	b.byIndex = x.byIndex
	return nil
}

// results decodes the outputs with the reference's error routing (minisched.go:50-75,
// ErrorFunc :283-298).
func (x *Ctx) results(b *HostBatch) []Result {
	out := make([]Result, len(b.pods))
	for j, pod := range b.pods {
		switch b.status[j] {
		case C.MSH_PLACED:
			out[j] = Result{Node: b.byIndex[b.idx[j]], Score: int64(b.score[j])}
		case C.MSH_FIT_ERROR:
			diag := framework.Diagnosis{NodeToStatusMap: framework.NodeToStatusMap{}, UnschedulablePlugins: sets.NewString()}
			if len(b.byIndex) > 0 { // some node failed NodeUnschedulable
				diag.UnschedulablePlugins.Insert("NodeUnschedulable")
			}
			out[j] = Result{FitErr: &framework.FitError{Pod: pod, Diagnosis: diag}} // as minisched.go:143-148
		default:
			out[j] = Result{Err: framework.AsStatus(framework.ErrNotFound).AsError()}
		}
	}
	return out
}

// ScheduleBatch runs minisched.go:50-87 for every pod against the uploaded snapshot, synchronously.
func (x *Ctx) ScheduleBatch(pods []*v1.Pod, b *HostBatch) ([]Result, error) {
	if !x.hasNodes {
		return nil, errors.New("gpusched: UploadNodes has not been called")
	}
	if err := x.pack(b, pods); err != nil {
		return nil, err
	}
	p := len(pods)
	if rc := C.msh_schedule_batch(x.c, C.int32_t(p), ptrI8(b.pd[:p]), ptrU8(b.pt[:p]), ptrI32(b.idx[:p]),
		ptrI64(b.score[:p]), ptrI32(b.status[:p])); rc != C.MSH_OK {
		return nil, x.lastErr("msh_schedule_batch", rc)
	}
	return x.results(b), nil
}

// Submit launches a batch asynchronously (msh_schedule_batch_async) and returns at once: the caller
// packs and submits the next drained batch into another HostBatch while this one runs. Collect it
// with Wait. Batches of one Ctx complete in submission order.
func (x *Ctx) Submit(pods []*v1.Pod, b *HostBatch) error {
	if !x.hasNodes {
		return errors.New("gpusched: UploadNodes has not been called")
	}
	if b.ticket != 0 {
		return errors.New("gpusched: HostBatch has a batch in flight; Wait for it first")
	}
	if err := x.pack(b, pods); err != nil {
		return err
	}
	p := len(pods)
	if rc := C.msh_schedule_batch_async(x.c, C.int32_t(p), ptrI8(b.pd[:p]), ptrU8(b.pt[:p]), ptrI32(b.idx[:p]),
		ptrI64(b.score[:p]), ptrI32(b.status[:p]), &b.ticket); rc != C.MSH_OK {
		b.ticket = 0
		return x.lastErr("msh_schedule_batch_async", rc)
	}
	return nil
}

// Wait returns the results of the batch last submitted into b.
func (x *Ctx) Wait(b *HostBatch) ([]Result, error) {
	if b.ticket == 0 {
		return nil, errors.New("gpusched: no batch in flight in this HostBatch")
	}
	t := b.ticket
	b.ticket = 0
	if rc := C.msh_wait(x.c, t); rc != C.MSH_OK {
		return nil, x.lastErr("msh_wait", rc)
	}
	return x.results(b), nil
}

// ScheduleSequential places the pods one at a time with a node-state commit between placements
// (the reference's serial Run loop, minisched.go:28-30, on the device). maxPodsPerNode > 0 makes a
// node infeasible once it holds that many pods (build extension); 0 = reference semantics, where no
// commit feeds a later decision: the library then runs the batch kernel and adds the placements to the
// node counts (a no-capacity shortcut with the serial loop's placements and counts).
func (x *Ctx) ScheduleSequential(pods []*v1.Pod, b *HostBatch, maxPodsPerNode int32) ([]Result, error) {
	if !x.hasNodes {
		return nil, errors.New("gpusched: UploadNodes has not been called")
	}
	if err := x.pack(b, pods); err != nil {
		return nil, err
	}
	p := len(pods)
	if rc := C.msh_schedule_sequential(x.c, C.int32_t(p), ptrI8(b.pd[:p]), ptrU8(b.pt[:p]), C.int32_t(maxPodsPerNode),
		ptrI32(b.idx[:p]), ptrI64(b.score[:p]), ptrI32(b.status[:p]), nil, nil); rc != C.MSH_OK {
		return nil, x.lastErr("msh_schedule_sequential", rc)
	}
	return x.results(b), nil
}

// ---- node sharding (ABI v8): the node table split over GPUs, the cross-shard merge inside the library ----
//
// The reference's selectHost keeps the first maximum of the whole List-order node list
// (minisched.go:304-325). Split into contiguous slices, each shard finds its own first maximum per pod,
// and the library merges them back into the global one: in one process over several devices (Group), or
// one process per GPU over an RCCL communicator (Ctx.InitComm + ScheduleNodeShard).

// sortedNodes is the List order of nodes (byte-sorted names, the apiserver's etcd key order).
func sortedNodes(nodes []v1.Node) []*v1.Node {
	sorted := make([]*v1.Node, len(nodes))
	for i := range nodes {
		sorted[i] = &nodes[i]
	}
	sort.Slice(sorted, func(a, b int) bool { return sorted[a].Name < sorted[b].Name })
	return sorted
}

// shardRange is the contiguous slice [lo, hi) of n List positions that shard k of w holds.
func shardRange(n, w, k int) (int, int) { return n * k / w, n * (k + 1) / w }

// uploadSlice uploads List positions [lo, hi) of sorted as x's table.
func (x *Ctx) uploadSlice(sorted []*v1.Node, lo, hi int) error {
	uns := make([]C.uint8_t, hi-lo)
	dig := make([]C.int8_t, hi-lo)
	for i, n := range sorted[lo:hi] {
		if n.Spec.Unschedulable {
			uns[i] = 1
		}
		dig[i] = C.int8_t(suffixDigit(n.Name))
	}
	if rc := C.msh_upload_nodes(x.c, C.int32_t(hi-lo), ptrU8(uns), ptrI8(dig)); rc != C.MSH_OK {
		return x.lastErr("msh_upload_nodes", rc)
	}
	x.hasNodes = true
	return nil
}

// Group is one scheduler process driving several GPUs (msh_group_*): shard k (a Ctx on devices[k])
// holds the k-th contiguous slice of the List order; msh_group_schedule_batch runs every shard's kernel
// on its own device and merges on devices[0], reading the shards' per-pod results over xGMI.
type Group struct {
	g       *C.msh_group
	shards  []*Ctx
	byIndex []*v1.Node // global List order
}

// NewGroup creates one shard Ctx per device (the same plugin lists on each) and the group over them.
func NewGroup(devices []int, filters []framework.FilterPlugin, preScores []framework.PreScorePlugin,
	scores []ScoreConfig) (*Group, error) {
	if len(devices) < 1 || len(devices) > C.MSH_GROUP_MAX_SHARDS {
		return nil, fmt.Errorf("gpusched: 1..%d devices", int(C.MSH_GROUP_MAX_SHARDS))
	}
	gr := &Group{}
	for _, d := range devices {
		x, err := New(d, filters, preScores, scores)
		if err != nil {
			gr.Close()
			return nil, err
		}
		gr.shards = append(gr.shards, x)
	}
	cs := make([]*C.msh_ctx, len(gr.shards)) // C memory holds no Go pointer: the handles are C pointers
	for k, x := range gr.shards {
		cs[k] = x.c
	}
	if rc := C.msh_group_create(&cs[0], C.int32_t(len(cs)), &gr.g); rc != C.MSH_OK {
		err := fmt.Errorf("msh_group_create: %d: %s", int(rc), C.GoString(C.msh_group_last_error(nil)))
		gr.Close()
		return nil, err
	}
	runtime.SetFinalizer(gr, (*Group).Close)
	return gr, nil
}

// Close releases the group, then its shard contexts.
func (gr *Group) Close() {
	if gr.g != nil {
		C.msh_group_destroy(gr.g)
		gr.g = nil
	}
	for _, x := range gr.shards {
		x.Close()
	}
	gr.shards = nil
	runtime.SetFinalizer(gr, nil)
}

// UploadNodes puts the nodes in List order and uploads slice k to shard k (replacing minisched.go:40).
func (gr *Group) UploadNodes(nodes []v1.Node) error {
	sorted := sortedNodes(nodes)
	for k, x := range gr.shards {
		lo, hi := shardRange(len(sorted), len(gr.shards), k)
		if err := x.uploadSlice(sorted, lo, hi); err != nil {
			return err
		}
	}
	gr.byIndex = sorted
	return nil
}

// ScheduleBatch runs minisched.go:50-87 for every pod against the whole (sharded) table, synchronously.
func (gr *Group) ScheduleBatch(pods []*v1.Pod, b *HostBatch) ([]Result, error) {
	if gr.byIndex == nil {
		return nil, errors.New("gpusched: UploadNodes has not been called")
	}
	x := &Ctx{byIndex: gr.byIndex} // packing and decoding against the global List order
	if err := x.pack(b, pods); err != nil {
		return nil, err
	}
	p := len(pods)
	if rc := C.msh_group_schedule_batch(gr.g, C.int32_t(p), ptrI8(b.pd[:p]), ptrU8(b.pt[:p]), ptrI32(b.idx[:p]),
		ptrI64(b.score[:p]), ptrI32(b.status[:p])); rc != C.MSH_OK {
		return nil, fmt.Errorf("msh_group_schedule_batch: %d: %s", int(rc), C.GoString(C.msh_group_last_error(gr.g)))
	}
	return x.results(b), nil
}

// CommID makes the id of a new RCCL communicator (msh_comm_unique_id): rank 0 calls it and ships the
// bytes to every rank (over the scheduler's own channel).
func CommID() ([]byte, error) {
	buf := make([]byte, C.MSH_COMM_ID_BYTES)
	if rc := C.msh_comm_unique_id((*C.uint8_t)(unsafe.Pointer(&buf[0]))); rc != C.MSH_OK {
		return nil, fmt.Errorf("msh_comm_unique_id: %d", int(rc))
	}
	return buf, nil
}

// InitComm joins x to the communicator `id` as rank `rank` of `world` (one process per GPU); it returns
// once every rank has joined.
func (x *Ctx) InitComm(id []byte, world, rank int) error {
	if len(id) != C.MSH_COMM_ID_BYTES {
		return fmt.Errorf("gpusched: a comm id is %d bytes", int(C.MSH_COMM_ID_BYTES))
	}
	cid := C.CBytes(id) // C memory: the library reads it during the call
	defer C.free(cid)
	if rc := C.msh_comm_init(x.c, (*C.uint8_t)(cid), C.int32_t(world), C.int32_t(rank)); rc != C.MSH_OK {
		return x.lastErr("msh_comm_init", rc)
	}
	return nil
}

// UploadNodeShard keeps the whole List order for decoding (every rank's informer holds every node) and
// uploads this rank's slice; it returns the slice's global base for ScheduleNodeShard.
func (x *Ctx) UploadNodeShard(nodes []v1.Node, world, rank int) (int64, error) {
	sorted := sortedNodes(nodes)
	lo, hi := shardRange(len(sorted), world, rank)
	if err := x.uploadSlice(sorted, lo, hi); err != nil {
		return 0, err
	}
	x.byIndex = sorted
	return int64(lo), nil
}

// ScheduleNodeShard is ScheduleBatch over the table split across the communicator's ranks
// (msh_schedule_nodeshard): every rank calls it with the same pods and gets every pod's decision.
func (x *Ctx) ScheduleNodeShard(pods []*v1.Pod, b *HostBatch, nodeBase int64) ([]Result, error) {
	if !x.hasNodes {
		return nil, errors.New("gpusched: UploadNodeShard has not been called")
	}
	if err := x.pack(b, pods); err != nil {
		return nil, err
	}
	p := len(pods)
	if rc := C.msh_schedule_nodeshard(x.c, C.int32_t(p), ptrI8(b.pd[:p]), ptrU8(b.pt[:p]), C.int64_t(nodeBase),
		ptrI32(b.idx[:p]), ptrI64(b.score[:p]), ptrI32(b.status[:p])); rc != C.MSH_OK {
		return nil, x.lastErr("msh_schedule_nodeshard", rc)
	}
	return x.results(b), nil
}

// suffixDigit is strconv.Atoi(name[len(name)-1:]) (nodenumber.go:51-56, :81-87): only '0'..'9' parse.
func suffixDigit(name string) int {
	if name == "" {
		return -1
	}
	c := name[len(name)-1]
	if c >= '0' && c <= '9' {
		return int(c - '0')
	}
	return -1
}

// tolerates is v1helper.TolerationsTolerateTaint(tolerations, unschedulable taint), what upstream
// NodeUnschedulable.Filter (k8s.io/kubernetes v1.22.0) asks.
func tolerates(ts []v1.Toleration) bool {
	taint := &v1.Taint{Key: v1.TaintNodeUnschedulable, Effect: v1.TaintEffectNoSchedule}
	for i := range ts {
		if ts[i].ToleratesTaint(taint) {
			return true
		}
	}
	return false
}

func ptrI32(s []C.int32_t) *C.int32_t {
	if len(s) == 0 {
		return nil
	}
	return &s[0]
}

func ptrI64(s []C.int64_t) *C.int64_t {
	if len(s) == 0 {
		return nil
	}
	return &s[0]
}

func ptrU8(s []C.uint8_t) *C.uint8_t {
	if len(s) == 0 {
		return nil
	}
	return &s[0]
}

func ptrI8(s []C.int8_t) *C.int8_t {
	if len(s) == 0 {
		return nil
	}
	return &s[0]
}
