package gpusched

// The Go comparison path of SURVEY.md §8(c): the reference's own plugins (upstream
// nodeunschedulable v1.22.0 and minisched's nodenumber), driven by a restatement of its plugin
// loops (RunFilterPlugins / RunPreScorePlugins / RunScorePlugins, minisched.go:115-199) with a
// first-max selectHost (the device's tie contract; minisched.go:304-325 reservoir-samples ties),
// against the device on the same snapshot: bit-exact node, score and status per pod.
// BenchmarkReferenceLoop is the Go CPU baseline (single goroutine, as the reference runs, and
// GOMAXPROCS-wide pod-parallel); BenchmarkDeviceBatch the C-ABI host-buffer call.
//
// Needs a GPU (msh_create fails with MSH_ERR_NO_DEVICE otherwise: the tests skip).

import (
	"context"
	"fmt"
	"math/rand"
	"runtime"
	"sync"
	"testing"

	"github.com/sanposhiho/mini-kube-scheduler/minisched/plugins/score/nodenumber"
	v1 "k8s.io/api/core/v1"
	metav1 "k8s.io/apimachinery/pkg/apis/meta/v1"
	"k8s.io/apimachinery/pkg/types"
	corelisters "k8s.io/client-go/listers/core/v1"
	"k8s.io/client-go/tools/cache"
	"k8s.io/kubernetes/pkg/scheduler/framework"
	"k8s.io/kubernetes/pkg/scheduler/framework/plugins/nodeunschedulable"
)

type refPlugins struct {
	filters   []framework.FilterPlugin
	preScores []framework.PreScorePlugin
	scores    []framework.ScorePlugin
}

func newRefPlugins(t testing.TB) refPlugins {
	nu, err := nodeunschedulable.New(nil, nil) // initialize.go:193-202
	if err != nil {
		t.Fatal(err)
	}
	nn, err := nodenumber.New(nil, nil) // initialize.go:204-213 (Permit's handle is not used here)
	if err != nil {
		t.Fatal(err)
	}
	return refPlugins{
		filters:   []framework.FilterPlugin{nu.(framework.FilterPlugin)},
		preScores: []framework.PreScorePlugin{nn.(framework.PreScorePlugin)},
		scores:    []framework.ScorePlugin{nn.(framework.ScorePlugin)},
	}
}

func newDevice(t testing.TB, rp refPlugins) *Ctx {
	scores := make([]ScoreConfig, len(rp.scores))
	for i, s := range rp.scores {
		scores[i] = ScoreConfig{Plugin: s, Weight: 1}
	}
	x, err := New(0, rp.filters, rp.preScores, scores)
	if err != nil {
		t.Skipf("no device: %v", err)
	}
	return x
}

type refResult struct {
	node   string
	score  int64
	status int // 0 placed, 1 FitError, 2 score error
}

// refScheduleOne is scheduleOne's selection part (minisched.go:50-87) over the List-ordered
// snapshot, with selectHost's first maximum.
func refScheduleOne(rp refPlugins, pod *v1.Pod, nodes []*v1.Node) refResult {
	ctx := context.Background()
	state := framework.NewCycleState()
	feasible := make([]*v1.Node, 0, len(nodes))
	for _, n := range nodes { // RunFilterPlugins, minisched.go:115-151
		ni := framework.NewNodeInfo()
		ni.SetNode(n)
		ok := true
		for _, pl := range rp.filters {
			if st := pl.Filter(ctx, state, pod, ni); !st.IsSuccess() {
				ok = false
				break
			}
		}
		if ok {
			feasible = append(feasible, n)
		}
	}
	if len(feasible) == 0 {
		return refResult{status: 1}
	}
	for _, pl := range rp.preScores { // RunPreScorePlugins, :153-162
		if st := pl.PreScore(ctx, state, pod, feasible); !st.IsSuccess() {
			return refResult{status: 2}
		}
	}
	total := make([]int64, len(feasible)) // RunScorePlugins, :164-199 (no normalize: NodeNumber has none)
	for i, n := range feasible {
		for _, pl := range rp.scores {
			s, st := pl.Score(ctx, state, pod, n.Name)
			if !st.IsSuccess() {
				return refResult{status: 2}
			}
			total[i] += s
		}
	}
	best := 0 // selectHost, :304-325, ties -> first
	for i := 1; i < len(total); i++ {
		if total[i] > total[best] {
			best = i
		}
	}
	return refResult{node: feasible[best].Name, score: total[best]}
}

// synthetic snapshot of SURVEY.md §8(d): node%d (List order = byte order), 10% unschedulable,
// pod%d with 1% non-digit suffixes and 5% tolerating the unschedulable taint.
func synth(n, p int, seed int64) ([]v1.Node, []*v1.Pod) {
	r := rand.New(rand.NewSource(seed))
	nodes := make([]v1.Node, n)
	for i := range nodes {
		nodes[i] = v1.Node{ObjectMeta: metav1.ObjectMeta{Name: fmt.Sprintf("node%d", i)},
			Spec: v1.NodeSpec{Unschedulable: r.Float64() < 0.10}}
	}
	pods := make([]*v1.Pod, p)
	for j := range pods {
		name := fmt.Sprintf("pod%d", j)
		if r.Float64() < 0.01 {
			name += "-x"
		}
		pod := &v1.Pod{ObjectMeta: metav1.ObjectMeta{Name: name, UID: types.UID(fmt.Sprintf("uid-%d", j))}}
		if r.Float64() < 0.05 {
			pod.Spec.Tolerations = []v1.Toleration{{Key: v1.TaintNodeUnschedulable, Operator: v1.TolerationOpExists,
				Effect: v1.TaintEffectNoSchedule}}
		}
		pods[j] = pod
	}
	return nodes, pods
}

func compare(t *testing.T, rp refPlugins, got []Result, pods []*v1.Pod, byIndex []*v1.Node) {
	t.Helper()
	for j, pod := range pods {
		want := refScheduleOne(rp, pod, byIndex)
		g := got[j]
		switch {
		case want.status == 1:
			if g.FitErr == nil {
				t.Fatalf("pod %s: want FitError, got %+v", pod.Name, g)
			}
		case want.status == 2:
			if g.Err == nil {
				t.Fatalf("pod %s: want a score error, got %+v", pod.Name, g)
			}
		default:
			if g.Node == nil || g.Node.Name != want.node || g.Score != want.score {
				t.Fatalf("pod %s: want %s (%d), got %+v", pod.Name, want.node, want.score, g)
			}
		}
	}
}

// The reference's own known answer (sched.go:70-143): nine unschedulable nodes -> FitError with
// UnschedulablePlugins {NodeUnschedulable}; after node10 is added, pod1 -> node10.
func TestReferenceScenario(t *testing.T) {
	rp := newRefPlugins(t)
	x := newDevice(t, rp)
	defer x.Close()
	nodes := make([]v1.Node, 0, 10)
	for i := 0; i < 9; i++ {
		nodes = append(nodes, v1.Node{ObjectMeta: metav1.ObjectMeta{Name: fmt.Sprintf("node%d", i)},
			Spec: v1.NodeSpec{Unschedulable: true}})
	}
	pod := &v1.Pod{ObjectMeta: metav1.ObjectMeta{Name: "pod1"}}
	b, err := NewHostBatch(16)
	if err != nil {
		t.Fatal(err)
	}
	if _, err := x.UploadNodes(nodes); err != nil {
		t.Fatal(err)
	}
	res, err := x.ScheduleBatch([]*v1.Pod{pod}, b)
	if err != nil {
		t.Fatal(err)
	}
	if res[0].FitErr == nil || !res[0].FitErr.Diagnosis.UnschedulablePlugins.Has("NodeUnschedulable") {
		t.Fatalf("want FitError{NodeUnschedulable}, got %+v", res[0])
	}
	nodes = append(nodes, v1.Node{ObjectMeta: metav1.ObjectMeta{Name: "node10"}})
	if _, err := x.UploadNodes(nodes); err != nil {
		t.Fatal(err)
	}
	res, err = x.ScheduleBatch([]*v1.Pod{pod}, b)
	if err != nil {
		t.Fatal(err)
	}
	if res[0].Node == nil || res[0].Node.Name != "node10" {
		t.Fatalf("want node10, got %+v", res[0])
	}
}

// BASELINE C2 (1k nodes x 10k pods): every pod bit-exact against the reference plugins; then a
// cordon flip through UpdateNode, and the async pair on two HostBatches.
func TestBatchMatchesReferencePlugins(t *testing.T) {
	rp := newRefPlugins(t)
	x := newDevice(t, rp)
	defer x.Close()
	nodes, pods := synth(1000, 10000, 0x6d696e69)
	byIndex, err := x.UploadNodes(nodes)
	if err != nil {
		t.Fatal(err)
	}
	b, err := NewHostBatch(len(pods))
	if err != nil {
		t.Fatal(err)
	}
	got, err := x.ScheduleBatch(pods, b)
	if err != nil {
		t.Fatal(err)
	}
	compare(t, rp, got, pods, byIndex)

	flipped := byIndex[17].DeepCopy()
	flipped.Spec.Unschedulable = !flipped.Spec.Unschedulable
	if err := x.UpdateNode(flipped); err != nil {
		t.Fatal(err)
	}
	b2, err := NewHostBatch(len(pods))
	if err != nil {
		t.Fatal(err)
	}
	if err := x.Submit(pods[:5000], b); err != nil {
		t.Fatal(err)
	}
	if err := x.Submit(pods[5000:], b2); err != nil {
		t.Fatal(err)
	}
	r1, err := x.Wait(b)
	if err != nil {
		t.Fatal(err)
	}
	r2, err := x.Wait(b2)
	if err != nil {
		t.Fatal(err)
	}
	compare(t, rp, append(r1, r2...), pods, x.byIndex)
}

// The informer path of batch.go (verdict r3 #6): nodes arrive through NodeSnapshot's handlers; a
// cordon flip between two batches (the Node Update handler, eventhandler.go:45-65) reaches the device
// as a patch, not a re-upload, and the second batch sees it; an Add then forces one upload. Mirrored
// on the Python side by tests/test_pipeline.py::test_node_cache_cordon_flip_between_batches_gpu.
func TestNodeSnapshotCordonFlipBetweenBatches(t *testing.T) {
	rp := newRefPlugins(t)
	x := newDevice(t, rp)
	defer x.Close()
	nodes, pods := synth(2000, 4000, 0x5eed)
	snap := NewNodeSnapshot()
	for i := range nodes {
		snap.OnAdd(&nodes[i])
	}
	if kind, err := snap.Sync(x); err != nil || kind != "upload" {
		t.Fatalf("first sync: %q %v", kind, err)
	}
	b, err := NewHostBatch(len(pods))
	if err != nil {
		t.Fatal(err)
	}
	got, err := x.ScheduleBatch(pods, b)
	if err != nil {
		t.Fatal(err)
	}
	compare(t, rp, got, pods, x.byIndex)
	if kind, _ := snap.Sync(x); kind != "clean" {
		t.Fatalf("no event: want clean, got %q", kind)
	}
	// cordon the first schedulable node of the List and uncordon the first unschedulable one
	var flips []*v1.Node
	for _, n := range x.byIndex {
		if (len(flips) == 0 && !n.Spec.Unschedulable) || (len(flips) == 1 && n.Spec.Unschedulable) {
			c := n.DeepCopy()
			c.Spec.Unschedulable = !c.Spec.Unschedulable
			snap.OnUpdate(n, c)
			flips = append(flips, c)
		}
	}
	if kind, err := snap.Sync(x); err != nil || kind != "patch" {
		t.Fatalf("cordon flip: want patch, got %q %v", kind, err)
	}
	got, err = x.ScheduleBatch(pods, b)
	if err != nil {
		t.Fatal(err)
	}
	compare(t, rp, got, pods, x.byIndex) // the reference loop over the updated snapshot
	snap.OnAdd(&v1.Node{ObjectMeta: metav1.ObjectMeta{Name: "node0000"}})
	if kind, err := snap.Sync(x); err != nil || kind != "upload" {
		t.Fatalf("add: want upload, got %q %v", kind, err)
	}
	got, err = x.ScheduleBatch(pods, b)
	if err != nil {
		t.Fatal(err)
	}
	compare(t, rp, got, pods, x.byIndex)
}

// The store has synced (WaitForCacheSync returned, scheduler.go:72-75) but the handlers have been
// called for only part of it (advisor r4): the first Sync of a lister-backed snapshot uploads the whole
// store, so the first batch matches the reference's per-cycle LIST; the late Adds then patch identical
// values, and the batch after them is unchanged.
func TestNodeSnapshotFirstSyncReadsTheStore(t *testing.T) {
	rp := newRefPlugins(t)
	x := newDevice(t, rp)
	defer x.Close()
	nodes, pods := synth(2000, 4000, 0x51)
	store := cache.NewIndexer(cache.MetaNamespaceKeyFunc, cache.Indexers{})
	for i := range nodes {
		if err := store.Add(&nodes[i]); err != nil {
			t.Fatal(err)
		}
	}
	snap := NewNodeSnapshotFromLister(corelisters.NewNodeLister(store))
	for i := 0; i < len(nodes)/3; i++ { // the handlers lag behind the store
		snap.OnAdd(&nodes[i])
	}
	if kind, err := snap.Sync(x); err != nil || kind != "upload" {
		t.Fatalf("first sync: %q %v", kind, err)
	}
	if len(x.byIndex) != len(nodes) {
		t.Fatalf("first upload holds %d of the store's %d nodes", len(x.byIndex), len(nodes))
	}
	b, err := NewHostBatch(len(pods))
	if err != nil {
		t.Fatal(err)
	}
	got, err := x.ScheduleBatch(pods, b)
	if err != nil {
		t.Fatal(err)
	}
	compare(t, rp, got, pods, x.byIndex)
	for i := len(nodes) / 3; i < len(nodes); i++ { // the late handler calls
		snap.OnAdd(&nodes[i])
	}
	if kind, err := snap.Sync(x); err != nil || kind != "patch" {
		t.Fatalf("late adds: want patch, got %q %v", kind, err)
	}
	again, err := x.ScheduleBatch(pods, b)
	if err != nil {
		t.Fatal(err)
	}
	for j := range got {
		if got[j].Node != again[j].Node && (got[j].Node == nil || again[j].Node == nil || got[j].Node.Name != again[j].Node.Name) {
			t.Fatalf("pod %d: %v before the late adds, %v after", j, got[j].Node, again[j].Node)
		}
	}
}

// An upload between Submit and Wait must not change how the batch in flight decodes (advisor r3):
// the launch read the table published at Submit, and Wait maps its indices through that table's nodes.
func TestWaitDecodesAgainstTheSubmittedTable(t *testing.T) {
	rp := newRefPlugins(t)
	x := newDevice(t, rp)
	defer x.Close()
	nodes, pods := synth(1000, 2000, 0x77)
	before, err := x.UploadNodes(nodes)
	if err != nil {
		t.Fatal(err)
	}
	b, err := NewHostBatch(len(pods))
	if err != nil {
		t.Fatal(err)
	}
	if err := x.Submit(pods, b); err != nil {
		t.Fatal(err)
	}
	if _, err := x.UploadNodes(nodes[:500]); err != nil { // a different table, published meanwhile
		t.Fatal(err)
	}
	got, err := x.Wait(b)
	if err != nil {
		t.Fatal(err)
	}
	compare(t, rp, got, pods, before)
}

func BenchmarkReferenceLoopC3(b *testing.B) {
	rp := newRefPlugins(b)
	nodes, pods := synth(5000, 2000, 0x6d696e69) // a bounded sample of the 100k-pod batch
	byIndex := make([]*v1.Node, len(nodes))
	for i := range nodes {
		byIndex[i] = &nodes[i]
	}
	b.Run("goroutines=1", func(b *testing.B) {
		for it := 0; it < b.N; it++ {
			for _, pod := range pods {
				refScheduleOne(rp, pod, byIndex)
			}
		}
		b.ReportMetric(float64(len(pods)*len(nodes)*b.N)/b.Elapsed().Seconds(), "pod-node-evals/s")
	})
	b.Run(fmt.Sprintf("goroutines=%d", runtime.GOMAXPROCS(0)), func(b *testing.B) {
		w := runtime.GOMAXPROCS(0)
		for it := 0; it < b.N; it++ {
			var wg sync.WaitGroup
			for k := 0; k < w; k++ {
				wg.Add(1)
				go func(k int) {
					defer wg.Done()
					for j := k; j < len(pods); j += w {
						refScheduleOne(rp, pods[j], byIndex)
					}
				}(k)
			}
			wg.Wait()
		}
		b.ReportMetric(float64(len(pods)*len(nodes)*b.N)/b.Elapsed().Seconds(), "pod-node-evals/s")
	})
}

func BenchmarkDeviceBatchC3(b *testing.B) {
	rp := newRefPlugins(b)
	x := newDevice(b, rp)
	defer x.Close()
	nodes, pods := synth(5000, 100000, 0x6d696e69)
	if _, err := x.UploadNodes(nodes); err != nil {
		b.Fatal(err)
	}
	hb, err := NewHostBatch(len(pods))
	if err != nil {
		b.Fatal(err)
	}
	b.ResetTimer()
	for it := 0; it < b.N; it++ {
		if _, err := x.ScheduleBatch(pods, hb); err != nil {
			b.Fatal(err)
		}
	}
	b.ReportMetric(float64(len(pods)*len(nodes)*b.N)/b.Elapsed().Seconds(), "pod-node-evals/s")
}
