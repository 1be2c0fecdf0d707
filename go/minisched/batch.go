package minisched

// The batched scheduling loop: scheduleOne's selection part (minisched.go:40-87) for a whole batch
// drained from activeQ, on the device through gpusched; Permit and Bind stay per pod, exactly as
// scheduleOne runs them (:89-112). The device's node table follows the Node informer
// (gpusched.NodeSnapshot: a cordon flip is an O(1) patch, an Add or a Delete one upload) instead of
// the per-cycle LIST (:40). Wire it in place of Run when the plugin lists are the device's:
//
//	snap := gpusched.NewNodeSnapshot()
//	informerFactory.Core().V1().Nodes().Informer().AddEventHandler(snap.Handlers()) // before Start
//	gpu, err := gpusched.New(0, sched.filterPlugins, sched.preScorePlugins, gpusched.Scores(sched.scorePlugins))
//	if errors.Is(err, gpusched.ErrUnsupported) { sched.Run(ctx) } else { sched.RunBatched(ctx, gpu, snap, 100000) }

import (
	"context"

	"github.com/sanposhiho/mini-kube-scheduler/minisched/gpusched"
	v1 "k8s.io/api/core/v1"
	"k8s.io/apimachinery/pkg/util/wait"
	"k8s.io/klog/v2"
	"k8s.io/kubernetes/pkg/scheduler/framework"
)

// RunBatched is Run (minisched.go:28-30) with batches of up to maxBatch pods per device call.
func (sched *Scheduler) RunBatched(ctx context.Context, gpu *gpusched.Ctx, snap *gpusched.NodeSnapshot, maxBatch int) {
	hb, err := gpusched.NewHostBatch(maxBatch)
	if err != nil {
		klog.Error(err)
		return
	}
	wait.UntilWithContext(ctx, func(ctx context.Context) { sched.scheduleBatch(ctx, gpu, snap, hb, maxBatch) }, 0)
}

func (sched *Scheduler) scheduleBatch(ctx context.Context, gpu *gpusched.Ctx, snap *gpusched.NodeSnapshot,
	hb *gpusched.HostBatch, maxBatch int) {
	pods := sched.SchedulingQueue.NextPods(maxBatch)
	// the informer's deltas since the last batch: a patch, an upload, or nothing (no LIST, :40)
	if _, err := snap.Sync(gpu); err != nil {
		klog.Error(err)
		for _, pod := range pods {
			sched.ErrorFunc(pod, err)
		}
		return
	}
	results, err := gpu.ScheduleBatch(pods, hb)
	if err != nil {
		klog.Error(err)
		for _, pod := range pods {
			sched.ErrorFunc(pod, err)
		}
		return
	}
	for j, r := range results {
		pod := pods[j]
		switch {
		case r.FitErr != nil:
			sched.ErrorFunc(pod, r.FitErr) // :50-55, UnschedulablePlugins kept for requeue
		case r.Err != nil:
			klog.Error(r.Err)
			sched.ErrorFunc(pod, nil) // :70-75 pass the filter's nil error
		default:
			sched.permitAndBind(ctx, pod, r.Node.Name)
		}
	}
}

// permitAndBind is scheduleOne's tail (:89-112), unchanged, for one placed pod.
func (sched *Scheduler) permitAndBind(ctx context.Context, pod *v1.Pod, nodename string) {
	state := framework.NewCycleState()
	status := sched.RunPermitPlugins(ctx, state, pod, nodename)
	if status.Code() != framework.Wait && !status.IsSuccess() {
		klog.Error(status.AsError())
		sched.ErrorFunc(pod, nil)
		return
	}
	go func() {
		status := sched.WaitOnPermit(ctx, pod)
		if !status.IsSuccess() {
			klog.Error(status.AsError())
			sched.ErrorFunc(pod, nil)
			return
		}
		if err := sched.Bind(ctx, nil, pod, nodename); err != nil {
			klog.Error(err)
			sched.ErrorFunc(pod, err)
			return
		}
		klog.Info("minischeduler: Bind Pod successfully")
	}()
}
