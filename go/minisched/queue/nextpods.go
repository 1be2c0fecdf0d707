package queue

// NextPods is the batch form of NextPod (queue.go:84-92): it waits until activeQ holds a pod (the
// reference busy-spins; this waits with a short sleep) and then drains up to max pods in FIFO
// order under the queue lock, so one device call schedules all of them (gpusched.Ctx.ScheduleBatch).
// Pods re-added while a batch is in flight land behind it, as with NextPod.

import (
	"time"

	v1 "k8s.io/api/core/v1"
)

func (s *SchedulingQueue) NextPods(max int) []*v1.Pod {
	if max <= 0 {
		return nil
	}
	for {
		s.lock.Lock()
		if n := len(s.activeQ); n > 0 {
			if n > max {
				n = max
			}
			out := make([]*v1.Pod, n)
			for i := 0; i < n; i++ {
				out[i] = s.activeQ[i].Pod
			}
			s.activeQ = s.activeQ[n:]
			s.lock.Unlock()
			return out
		}
		s.lock.Unlock()
		time.Sleep(100 * time.Microsecond)
	}
}
