// export_mirt.go — accessor for the GPU worker (new file in the reference's shared/colour).
// Uncompiled here: this image has no Go toolchain (see go/README.md).
package colour

// Floats returns the colour's normalised channels (colour.go:16-19), which the GPU worker
// passes to libmirt unchanged: materials and lights reach the worker already quantized to
// uint8/255 by MarshalBinary (colour.go:64-83), and the kernels take them as given.
func (rgb RGB) Floats() [3]float64 {
	return [3]float64{rgb.r, rgb.g, rgb.b}
}
