// Command gpu is the drop-in GPU worker: the registration loop, the gRPC Trace server and
// the idle shutdown of worker/distributed/main.go:101-185, unchanged, with the per-pixel
// loop of BulkTrace (main.go:67-89) replaced by one libmirt call (package gpu).  The master,
// the pool and the registrar see an ordinary worker (shared/comms/comms.proto:20-47).
//
//   gpu <master address:port> <work order port> [GPU index | all | i,j,...]
//
// With "all" (or a list of indices) ONE worker serves every order on several GPUs of the box
// (gpu.NewBox: the order is cut into 8-px column strips dealt over the GPUs and assembled
// over RCCL), so the master's partition sees a single worker for the box.
//
// Uncompiled here: this image has no Go toolchain (go/README.md).  worker_c/mirt_worker.c
// runs the same library call sequence in C and tests/test_c_worker.py checks its frames.
package main

import (
	"bytes"
	"context"
	"encoding/gob"
	"fmt"
	"log"
	"net"
	"errors"
	"os"
	"strconv"
	"strings"
	"time"

	"github.com/golang/protobuf/ptypes/empty"
	"github.com/mwindels/distributed-raytracer/shared/comms"
	"github.com/mwindels/distributed-raytracer/shared/state"
	"github.com/mwindels/distributed-raytracer/worker/shared/gpu"
	"google.golang.org/grpc"
)

// registerFrequency and traceTimeout as in worker/distributed/main.go:20-24 (milliseconds).
const registerFrequency uint = 500
const traceTimeout uint = 2000

// Tracer implements comms.TraceServer (worker/distributed/main.go:27-32) on a GPU.
type Tracer struct {
	scene                     state.Environment
	screenWidth, screenHeight uint
	resetTraceTimeout         chan struct{}
	gpu                       *gpu.Worker
}

// timeoutReset as worker/distributed/main.go:35-43.
func (t *Tracer) timeoutReset() {
	defer func() {
		recover()
	}()
	t.resetTraceTimeout <- struct{}{}
}

// BulkTrace traces a work order (worker/distributed/main.go:46-91): decode the frame's
// diff, trace the rectangle on the GPU, return the colours column-major (i*height + j).
func (t *Tracer) BulkTrace(ctx context.Context, req *comms.WorkOrder) (*comms.TraceResults, error) {
	t.timeoutReset()
	x, y := int(req.GetX()), int(req.GetY())
	width, height := int(req.GetWidth()), int(req.GetHeight())
	results := &comms.TraceResults{Results: make([]*comms.TraceResults_Colour, width*height, width*height)}

	// The frame's mutable state (main.go:57-65).  Without a diff the reference's pixel loop
	// would call tracer.Trace on a zero EnvMutables, whose nil Objs R-tree tracer.go:32
	// dereferences (a panic that ends the worker process; the master would then time the
	// order out).  This worker answers such an order with black pixels instead: the one
	// place where its behaviour differs, and only for an order no master sends
	// (master/main.go:130-150 always attaches the frame's diff).
	var diff state.EnvMutables
	env := &diff
	if req.GetDiff() != nil {
		if err := gob.NewDecoder(bytes.NewBuffer(req.GetDiff())).Decode(&diff); err != nil {
			return nil, err
		}
		diff.LinkTo(t.scene)
	}
	var rgb8 []uint8
	if env.Objs != nil {
		var err error
		rgb8, err = t.gpu.BulkTrace(ctx, t.scene, env, x, y, width, height, int(t.screenWidth), int(t.screenHeight))
		if err != nil {
			if ctx.Err() == context.Canceled {
				return nil, ctx.Err()
			}
			return nil, err
		}
	}
	for k := range results.Results {
		c := &comms.TraceResults_Colour{}
		if rgb8 != nil {
			c.R, c.G, c.B = uint32(rgb8[3*k]), uint32(rgb8[3*k+1]), uint32(rgb8[3*k+2])
		}
		results.Results[k] = c
	}
	return results, nil
}

// Heartbeat as worker/distributed/main.go:94-98.
func (t *Tracer) Heartbeat(ctx context.Context, req *empty.Empty) (*empty.Empty, error) {
	t.timeoutReset()
	return &empty.Empty{}, nil
}

// register as worker/distributed/main.go:101-129, then the scene's meshes go to the GPU
// once (they are immutable for the worker's life).
func register(registerAddr string, listenPort uint32, w *gpu.Worker) (Tracer, error) {
	conn, err := grpc.Dial(registerAddr, grpc.WithInsecure())
	if err != nil {
		return Tracer{}, err
	}
	defer conn.Close()
	client := comms.NewRegistrationClient(conn)
	stateMsg, err := client.Register(context.Background(), &comms.WorkerLink{Port: listenPort})
	if err != nil {
		return Tracer{}, err
	}
	var newScene state.Environment
	if stateMsg.GetState() != nil {
		if err = gob.NewDecoder(bytes.NewBuffer(stateMsg.GetState())).Decode(&newScene); err != nil {
			return Tracer{}, err
		}
	} else {
		return Tracer{}, fmt.Errorf("No scene data recieved.")
	}
	if err = w.UploadScene(newScene); err != nil {
		return Tracer{}, err
	}
	return Tracer{scene: newScene, screenWidth: uint(stateMsg.GetScreenWidth()),
		screenHeight: uint(stateMsg.GetScreenHeight()), resetTraceTimeout: make(chan struct{}), gpu: w}, nil
}

func main() {
	if len(os.Args) != 3 && len(os.Args) != 4 {
		log.Fatalln("Improper parameters.  This program requires the parameters:" +
			"\n\t(1) master address (including port)" +
			"\n\t(2) work order listening port" +
			"\n\t(3) optional: GPU index (default 0), \"all\", or a comma-separated list of GPU indices")
	}
	masterAddr := os.Args[1]
	orderPort, err := strconv.ParseUint(os.Args[2], 10, 32)
	if err != nil {
		log.Fatalf("Could not parse port number \"%s\": %v.\n", os.Args[2], err)
	}
	devices := []int{0}
	if len(os.Args) == 4 {
		devices = nil
		if os.Args[3] == "all" {
			for d := 0; d < gpu.DeviceCount(); d++ {
				devices = append(devices, d)
			}
			if len(devices) == 0 {
				log.Fatalln("No GPU is visible.")
			}
		} else {
			for _, f := range strings.Split(os.Args[3], ",") {
				d, err := strconv.Atoi(f)
				if err != nil {
					log.Fatalf("Could not parse GPU index \"%s\": %v.\n", f, err)
				}
				devices = append(devices, d)
			}
		}
	}

	// One GPU context (or box) for the process's life (it sets up the device workspaces and
	// streams once).  While a device is busy or out of memory the worker keeps retrying, as
	// the reference keeps retrying its registration (worker/distributed/main.go:131-185); an
	// error that cannot go away (no such GPU, a library built for another GPU) ends it.
	var w *gpu.Worker
	for {
		if len(devices) == 1 {
			w, err = gpu.New(devices[0])
		} else {
			w, err = gpu.NewBox(devices)
		}
		if err == nil {
			break
		}
		var me *gpu.Error
		if !errors.As(err, &me) || !me.Transient() {
			log.Fatalf("GPU(s) %v: %v.\n", devices, err)
		}
		log.Printf("GPU(s) %v: %v (retrying).\n", devices, err)
		time.Sleep(time.Millisecond * time.Duration(registerFrequency))
	}
	defer w.Close()

	for {
		// a failed registration costs one RPC; only a successful one uploads meshes
		tracer, err := register(masterAddr, uint32(orderPort), w)
		if err == nil {
			server := grpc.NewServer()
			comms.RegisterTraceServer(server, &tracer)
			listener, err := net.Listen("tcp", fmt.Sprintf(":%d", orderPort))
			if err != nil {
				log.Fatalf("Failed to listen on port \"%d\": %v.\n", orderPort, err)
			}
			// close the trace server when no order or heartbeat arrives in time (main.go:157-169)
			go func() {
				for {
					select {
					case <-tracer.resetTraceTimeout:
					case <-time.After(time.Millisecond * time.Duration(traceTimeout)):
						close(tracer.resetTraceTimeout)
						server.GracefulStop()
						return
					}
				}
			}()
			if err = server.Serve(listener); err != nil {
				log.Printf("Tracer interrupted: %v.\n", err)
			} else {
				log.Printf("Tracer timed out after recieving no orders or heartbeats.\n")
			}
		} else {
			log.Printf("Failed to register: %v.\n", err)
		}
		// the next registration may bring another scene: drop this one's meshes
		w.ReleaseMeshes()
		time.Sleep(time.Millisecond * time.Duration(registerFrequency))
	}
}
